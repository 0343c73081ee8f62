#pragma once
// Drop-in for the reference's he::util (include/he_util.h:6-78) over hecdna types: the chain-index helpers and the
// level-dropping loops he::math and the least-squares demo use (src/core/he_math.cpp:224,
// src/demos/matrix_operations.cpp:995).  A level is dropped as the reference drops it: the constant 1 encoded at
// the ciphertext's parms_id and scale (CKKSEncoder::encode(double, parms_id, scale, pt), hec_encode_scalar), a
// multiply_plain, then rescale_to_next, so the scale follows SEAL's bookkeeping bit for bit.
#include <concepts>
#include <cstdint>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "hecdna/seal_compat.hpp"

namespace he::util
{
    // seal::util::uint_to_hex_string(&value, 1): upper-case hex digits without leading zeros ("0" for zero)
    inline std::string uint64_to_hex_string(std::uint64_t value)
    {
        static const char digits[] = "0123456789ABCDEF";
        std::string s;
        do {
            s.insert(s.begin(), digits[value & 15]);
            value >>= 4;
        } while (value);
        return s;
    }

    // ctx.get_context_data(ct.parms_id())->chain_index() (he_util.h:13-16)
    inline std::size_t get_chain_index(const hecdna::Context &ctx, const hecdna::Ciphertext &ct)
    {
        const auto cd = ctx.get_context_data(ct.parms_id());
        if (!cd) throw std::invalid_argument("encrypted is not valid for encryption parameters");
        return cd->chain_index();
    }

    // the same from EncryptionParameters (he_util.h:18-21): the chain is recomputed on the host from the parameters'
    // parms_ids, without a device context
    inline std::size_t get_chain_index(const hecdna::EncryptionParameters &parms, const hecdna::Ciphertext &ct)
    {
        const auto &q = parms.coeff_modulus();
        const hecdna::parms_id_type id = ct.parms_id();
        for (std::size_t l = 1; l <= q.size(); ++l)
            if (hecdna::compute_parms_id(parms.poly_modulus_degree(), q.data(), l) == id) return l - 1;
        throw std::invalid_argument("encrypted is not valid for encryption parameters");
    }

    // one Ciphertext, or a vector of Ciphertext pointers that share a level and scale (he_util.h:23-25)
    template <typename T>
    concept vectorCiphertextPtr_tn = std::same_as<std::decay_t<T>, hecdna::Ciphertext> ||
                                     std::same_as<std::decay_t<T>, std::vector<hecdna::Ciphertext *>>;

    namespace detail
    {
        template <vectorCiphertextPtr_tn T>
        const hecdna::Ciphertext &front(const T &cts)
        {
            if constexpr (std::is_same_v<std::decay_t<T>, hecdna::Ciphertext>) return cts;
            else return *cts[0];
        }
        template <vectorCiphertextPtr_tn T, class F>
        void each(T &cts, F &&f)
        {
            if constexpr (std::is_same_v<std::decay_t<T>, hecdna::Ciphertext>) f(cts);
            else
                for (hecdna::Ciphertext *c : cts) f(*c);
        }
    } // namespace detail

    // drop num_of_levels levels: per level, 1 is encoded at the (first) ciphertext's parms_id and scale once, and every
    // ciphertext is multiplied by it and rescaled (he_util.h:27-48)
    template <vectorCiphertextPtr_tn T>
    inline void drop_chain_levels(const hecdna::Context &ctx, const hecdna::CKKSEncoder &cencd, const hecdna::Evaluator &eval,
                                  hecdna::Plaintext &one_pt, T &&res_ct, std::size_t num_of_levels)
    {
        (void)ctx;
        for (std::size_t k = 0; k < num_of_levels; ++k) {
            const hecdna::Ciphertext &lead = detail::front(res_ct);
            cencd.encode(1.0, lead.parms_id(), lead.scale(), one_pt);
            detail::each(res_ct, [&](hecdna::Ciphertext &c) {
                eval.multiply_plain_inplace(c, one_pt);
                eval.rescale_to_next_inplace(c);
            });
        }
    }

    template <vectorCiphertextPtr_tn T>
    inline void drop_chain_levels(const hecdna::Context &ctx, const hecdna::CKKSEncoder &cencd, const hecdna::Evaluator &eval,
                                  T &&res_ct, std::size_t num_of_levels)
    {
        hecdna::Plaintext one_pt;
        drop_chain_levels(ctx, cencd, eval, one_pt, std::forward<T>(res_ct), num_of_levels);
    }

    // drop the ciphertext(s) to the chain index of to_reach_ct (he_util.h:57-70); the difference is taken in size_t,
    // as the reference takes it
    template <vectorCiphertextPtr_tn T>
    inline void reach_chain_level(const hecdna::Context &ctx, const hecdna::CKKSEncoder &cencd, const hecdna::Evaluator &eval,
                                  hecdna::Plaintext &one_pt, T &&res_ct, const hecdna::Ciphertext &to_reach_ct)
    {
        const std::size_t n = get_chain_index(ctx, detail::front(res_ct)) - get_chain_index(ctx, to_reach_ct);
        drop_chain_levels(ctx, cencd, eval, one_pt, std::forward<T>(res_ct), n);
    }

    template <vectorCiphertextPtr_tn T>
    inline void reach_chain_level(const hecdna::Context &ctx, const hecdna::CKKSEncoder &cencd, const hecdna::Evaluator &eval,
                                  T &&res_ct, const hecdna::Ciphertext &to_reach_ct)
    {
        hecdna::Plaintext one_pt;
        reach_chain_level(ctx, cencd, eval, one_pt, std::forward<T>(res_ct), to_reach_ct);
    }
} // namespace he::util
