// he::math over hecdna (reference src/core/he_math.cpp:22-269).  The iterations are written with the
// hecdna::Evaluator members the reference's he::operators forward to; the order of every encode, product,
// relinearization and rescale is the reference's, which is what fixes the output bits (CKKS rescaling rounds, so a
// reordered schedule would be a different ciphertext).  Constants are encoded with CKKSEncoder::encode(double,
// parms_id, scale) at the level and scale of the ciphertext they meet, as the reference encodes them.
#include "he_math.h"

#include <cassert>
#include <cmath>

#include "he_util.h"

using hecdna::Ciphertext;
using hecdna::CKKSEncoder;
using hecdna::Evaluator;
using hecdna::Plaintext;
using hecdna::RelinKeys;

namespace he::math
{
    namespace
    {
        // ct <- rescale(ct (x) encode(c, ct.parms_id, ct.scale))
        void times_const(const CKKSEncoder &cencd, const Evaluator &eval, Ciphertext &ct, double c, Plaintext &pt)
        {
            cencd.encode(c, ct.parms_id(), ct.scale(), pt);
            eval.multiply_plain_inplace(ct, pt);
            eval.rescale_to_next_inplace(ct);
        }
        // ct <- rescale(relin(ct (x) other)); other == nullptr squares
        void times_ct(const Evaluator &eval, const RelinKeys &rk, Ciphertext &ct, const Ciphertext *other)
        {
            if (other) eval.multiply_inplace(ct, *other);
            else eval.square_inplace(ct);
            eval.relinearize_inplace(ct, rk);
            eval.rescale_to_next_inplace(ct);
        }
    } // namespace

    // 1/x = a prod_k (1 + (1 - a x)^(2^k)), started from 2a - a^2 x (he_math.cpp:22-90)
    Ciphertext signed_inv(const CKKSEncoder &cencd, const Evaluator &eval, const RelinKeys &rk, const Ciphertext &x_ct,
                          double a, std::size_t iter_num)
    {
        assert(iter_num > 0);
        Plaintext pt;
        // y = -a^2 x, rescaled, + 2a
        cencd.encode(-a * a, x_ct.parms_id(), x_ct.scale(), pt);
        Ciphertext y_ct;
        eval.multiply_plain(x_ct, pt, y_ct);
        eval.rescale_to_next_inplace(y_ct);
        cencd.encode(2 * a, y_ct.parms_id(), y_ct.scale(), pt);
        eval.add_plain_inplace(y_ct, pt);
        if (iter_num == 1) return y_ct;

        // e = a x - 1, rescaled (the 1 encoded at e's level and scale)
        cencd.encode(a, x_ct.parms_id(), x_ct.scale(), pt);
        Ciphertext e_ct;
        eval.multiply_plain(x_ct, pt, e_ct);
        eval.rescale_to_next_inplace(e_ct);
        Plaintext one_pt;
        cencd.encode(1.0, e_ct.parms_id(), e_ct.scale(), one_pt);
        eval.sub_plain_inplace(e_ct, one_pt);
        // y drops one level with that same plaintext 1
        eval.multiply_plain_inplace(y_ct, one_pt);
        eval.rescale_to_next_inplace(y_ct);

        Ciphertext term_ct;
        for (std::size_t i = 1; i < iter_num; ++i) {
            times_ct(eval, rk, e_ct, nullptr);  // e^2
            cencd.encode(1.0, e_ct.parms_id(), e_ct.scale(), one_pt);
            eval.add_plain(e_ct, one_pt, term_ct);  // e^2 + 1
            times_ct(eval, rk, y_ct, &term_ct);
        }
        return y_ct;
    }

    // Newton for 1/sqrt(2x): y' = 3/2 y - x y^3, two levels per step (he_math.cpp:95-164, the `#if 1` form)
    Ciphertext inv_sqrt_twice(const CKKSEncoder &cencd, const Evaluator &eval, const RelinKeys &rk, const Ciphertext &x_ct,
                              double a, std::size_t iter_num)
    {
        assert(iter_num > 0);
        Ciphertext x_lvl = x_ct;  // x, dropped alongside the iterate
        const double y0 = a;
        Plaintext pt;
        // first step on the scalar y0: y = x (-y0^3), rescaled, + 3/2 y0
        cencd.encode(-y0 * y0 * y0, x_lvl.parms_id(), x_lvl.scale(), pt);
        Ciphertext y_ct;
        eval.multiply_plain(x_lvl, pt, y_ct);
        eval.rescale_to_next_inplace(y_ct);
        cencd.encode(3.0 / 2 * y0, y_ct.parms_id(), y_ct.scale(), pt);
        eval.add_plain_inplace(y_ct, pt);

        Ciphertext xy_ct, yp_ct;
        for (std::size_t i = 1; i < iter_num; ++i) {
            yp_ct = y_ct;
            times_const(cencd, eval, y_ct, 3.0 / 2, pt);  // 3/2 y
            times_const(cencd, eval, y_ct, 1.0, pt);      // one more level, to meet x y^3
            for (std::size_t j = 0; j < (i > 1 ? 2u : 1u); ++j) times_const(cencd, eval, x_lvl, 1.0, pt);
            eval.multiply(x_lvl, yp_ct, xy_ct);  // x y
            eval.relinearize_inplace(xy_ct, rk);
            eval.rescale_to_next_inplace(xy_ct);
            times_ct(eval, rk, yp_ct, nullptr);  // y^2
            times_ct(eval, rk, yp_ct, &xy_ct);   // x y^3
            eval.sub_inplace(y_ct, yp_ct);
        }
        return y_ct;
    }

    // sqrt(x) = (1/sqrt(2x)) (sqrt(2) x) (he_math.cpp:211-232)
    Ciphertext sqrt(const hecdna::Context &ctx, const CKKSEncoder &cencd, const Evaluator &eval, const RelinKeys &rk,
                    const Ciphertext &x_ct, double a, std::size_t iter_num)
    {
        Ciphertext y_ct = inv_sqrt_twice(cencd, eval, rk, x_ct, 1 / a / std::sqrt(2), iter_num);
        Plaintext pt;
        cencd.encode(std::sqrt(2), x_ct.parms_id(), x_ct.scale(), pt);
        Ciphertext s_ct;
        eval.multiply_plain(x_ct, pt, s_ct);
        eval.rescale_to_next_inplace(s_ct);
        he::util::reach_chain_level(ctx, cencd, eval, pt, s_ct, y_ct);
        times_ct(eval, rk, y_ct, &s_ct);
        return y_ct;
    }

    // |x| = (1/(sqrt(2)|x|)) (sqrt(2) x^2) (he_math.cpp:237-269)
    Ciphertext abs(const hecdna::Context &ctx, const CKKSEncoder &cencd, const Evaluator &eval, const RelinKeys &rk,
                   const Ciphertext &x_ct, double a, std::size_t iter_num)
    {
        Ciphertext sq_ct;
        eval.square(x_ct, sq_ct);
        eval.relinearize_inplace(sq_ct, rk);
        eval.rescale_to_next_inplace(sq_ct);
        Ciphertext y_ct = inv_sqrt_twice(cencd, eval, rk, sq_ct, 1 / a / std::sqrt(2), iter_num);
        Plaintext pt;
        times_const(cencd, eval, sq_ct, std::sqrt(2), pt);
        const std::size_t drops = ctx.get_context_data(sq_ct.parms_id())->chain_index() -
                                  ctx.get_context_data(y_ct.parms_id())->chain_index();
        for (std::size_t i = 0; i < drops; ++i) times_const(cencd, eval, sq_ct, 1.0, pt);
        times_ct(eval, rk, y_ct, &sq_ct);
        return y_ct;
    }
} // namespace he::math
