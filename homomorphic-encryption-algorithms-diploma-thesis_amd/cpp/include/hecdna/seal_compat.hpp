// hecdna C++ host API: RAII value types over the C-ABI (include/hecdna.h) that stand in for the
// seal:: types the reference's he_operators / he_linalg layer is written against
// (reference include/he_operators.h:3, include/he_linalg.h:4 include "seal/seal.h").
//
//   seal::SEALContext + EncryptionParameters  -> hecdna::Context
//   seal::Evaluator                           -> hecdna::Evaluator  (same member names, const)
//   seal::Ciphertext / Plaintext              -> hecdna::Ciphertext / Plaintext (value semantics,
//                                                copy = deep device copy, like SEAL)
//   seal::RelinKeys / GaloisKeys              -> hecdna::RelinKeys / GaloisKeys
//   seal::CoeffModulus::Create                -> hecdna::CoeffModulus::Create
//   seal::CKKSEncoder::encode                 -> hecdna::CKKSEncoder::encode (on the GPU, hec_encode /
//                                                hec_encode_scalar; a parms_id or a level selects the level)
//   seal::parms_id_type, get_context_data(...) -> hecdna::parms_id_type (BLAKE2b-256 of {scheme, N, the level's
//      ->chain_index()                            moduli}, SEAL's parms_id), hecdna::ContextData
//
// Errors are rethrown with SEAL's exception types and messages (std::invalid_argument,
// std::logic_error); HIP failures as std::runtime_error.  Objects live on the context's GPU.
#pragma once

#include <array>
#include <complex>
#include <cstddef>
#include <cstdint>
#include <ios>
#include <map>
#include <memory>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "hecdna.h"

namespace hecdna {

inline void check(int rc)
{
    if (rc == HEC_OK) return;
    const std::string msg = hec_last_error();
    if (rc == HEC_EINVAL) throw std::invalid_argument(msg);
    if (rc == HEC_ELOGIC) throw std::logic_error(msg);
    throw std::runtime_error(msg);
}

struct CoeffModulus {
    static std::vector<std::uint64_t> Create(std::size_t poly_modulus_degree, const std::vector<int> &bit_sizes)
    {
        std::vector<std::uint64_t> out(bit_sizes.size());
        check(hec_create_coeff_modulus(poly_modulus_degree, bit_sizes.data(), bit_sizes.size(), out.data()));
        return out;
    }
};

// seal::compr_mode_type and the byte type of SEAL's buffer load/save overloads
enum class compr_mode_type : std::uint8_t { none = HEC_COMPR_NONE, zlib = HEC_COMPR_ZLIB, zstd = HEC_COMPR_ZSTD };
using seal_byte = std::byte;

inline void seal_check(int rc)
{
    if (rc == HEC_EINVAL) throw std::invalid_argument(hec_seal_last_error());
    if (rc != HEC_OK) throw std::logic_error(hec_seal_last_error());
}

// seal::EncryptionParameters (CKKS): the SEAL wire format load/save (server.cpp:110-112, client.cpp:82)
class EncryptionParameters {
public:
    EncryptionParameters() = default;
    EncryptionParameters(std::size_t poly_modulus_degree, std::vector<std::uint64_t> coeff_modulus)
        : n_(poly_modulus_degree), q_(std::move(coeff_modulus)) {}
    std::size_t poly_modulus_degree() const { return n_; }
    const std::vector<std::uint64_t> &coeff_modulus() const { return q_; }
    void set_poly_modulus_degree(std::size_t n) { n_ = n; }
    void set_coeff_modulus(std::vector<std::uint64_t> q) { q_ = std::move(q); }
    std::streamoff load(const seal_byte *in, std::size_t size)
    {
        std::uint64_t n = 0, k = 0, used = 0;
        seal_check(hec_seal_parms_load(in, size, &n, nullptr, 0, &k, &used));
        q_.resize(k);
        seal_check(hec_seal_parms_load(in, size, &n, q_.data(), k, &k, &used));
        n_ = n;
        return (std::streamoff)used;
    }
    std::streamoff save(std::ostream &out, compr_mode_type mode = compr_mode_type::zstd) const
    {
        std::uint64_t w = 0;
        seal_check(hec_seal_parms_save(n_, q_.data(), q_.size(), (int)mode, nullptr, 0, &w));
        std::vector<char> b(w);
        seal_check(hec_seal_parms_save(n_, q_.data(), q_.size(), (int)mode, b.data(), w, &w));
        out.write(b.data(), (std::streamsize)w);
        return (std::streamoff)w;
    }

private:
    std::size_t n_ = 0;
    std::vector<std::uint64_t> q_;
};

// seal::parms_id_type: the BLAKE2b-256 hash of a level's EncryptionParameters (EncryptionParameters::compute_parms_id
// over {scheme, N, the level's coeff_modulus, plain modulus}); the same words SEAL writes in a ciphertext's header
using parms_id_type = std::array<std::uint64_t, 4>;
inline parms_id_type compute_parms_id(std::size_t N, const std::uint64_t *moduli, std::size_t count)
{
    parms_id_type id{};
    seal_check(hec_seal_parms_id(N, moduli, count, id.data()));
    return id;
}

// seal::SEALContext::ContextData of one level of the modulus switching chain.  A level keeps its first
// `coeff_modulus_size` primes; chain_index() counts the levels below it (the key level, all K primes, has the
// largest index K - 1; the last data level, one prime, has 0), as SEAL numbers its chain.
class ContextData {
public:
    ContextData(std::size_t level, std::size_t N, std::vector<std::uint64_t> moduli, parms_id_type id,
                std::shared_ptr<const ContextData> next)
        : level_(level), parms_(N, std::move(moduli)), id_(id), next_(std::move(next)) {}
    std::size_t chain_index() const { return level_ - 1; }
    const parms_id_type &parms_id() const { return id_; }
    const EncryptionParameters &parms() const { return parms_; }
    std::size_t coeff_modulus_size() const { return level_; }
    int total_coeff_modulus_bit_count() const
    {
        int bits = 0;
        for (std::uint64_t q : parms_.coeff_modulus()) bits += 64 - __builtin_clzll(q);
        return bits;
    }
    // the next level down the chain (nullptr below the last one), as SEAL's next_context_data()
    std::shared_ptr<const ContextData> next_context_data() const { return next_; }

private:
    std::size_t level_;
    EncryptionParameters parms_;
    parms_id_type id_;
    std::shared_ptr<const ContextData> next_;
};

class Context {
public:
    // SEALContext ctx(parms) (server.cpp:112)
    explicit Context(const EncryptionParameters &parms, int device = 0)
        : Context(parms.poly_modulus_degree(), parms.coeff_modulus(), device) {}
    Context(std::size_t poly_modulus_degree, const std::vector<std::uint64_t> &coeff_modulus, int device = 0)
    {
        hec_context *c = nullptr;
        check(hec_context_create(poly_modulus_degree, coeff_modulus.data(), coeff_modulus.size(), device, &c));
        h_.reset(c, [](hec_context *p) { hec_context_destroy(p); });
        moduli_ = coeff_modulus;
        // the modulus switching chain, last level first: level l holds q_0 .. q_{l-1}; the key level all K primes
        std::shared_ptr<const ContextData> next;
        levels_.resize(coeff_modulus.size() + 1);
        for (std::size_t l = 1; l <= coeff_modulus.size(); ++l) {
            std::vector<std::uint64_t> q(coeff_modulus.begin(), coeff_modulus.begin() + (std::ptrdiff_t)l);
            const parms_id_type id = compute_parms_id(poly_modulus_degree, q.data(), l);
            // every level links to the one below, the key level too: SEAL's key_context_data()->next_context_data()
            // is first_context_data()
            auto cd = std::make_shared<const ContextData>(l, poly_modulus_degree, std::move(q), id, next);
            by_id_[id] = l;
            levels_[l] = cd;
            next = cd;
        }
    }
    hec_context *get() const { return h_.get(); }
    // SEALContext::get_context_data(parms_id): nullptr for an unknown parms_id (SEAL returns an empty pointer)
    std::shared_ptr<const ContextData> get_context_data(const parms_id_type &id) const
    {
        const auto it = by_id_.find(id);
        return it == by_id_.end() ? nullptr : levels_[it->second];
    }
    std::shared_ptr<const ContextData> key_context_data() const { return levels_.back(); }
    std::shared_ptr<const ContextData> first_context_data() const { return levels_[moduli_.size() - 1]; }
    std::shared_ptr<const ContextData> last_context_data() const { return levels_[1]; }
    const parms_id_type &key_parms_id() const { return levels_.back()->parms_id(); }
    const parms_id_type &first_parms_id() const { return first_context_data()->parms_id(); }
    const parms_id_type &last_parms_id() const { return levels_[1]->parms_id(); }
    // the level (number of primes) of a parms_id; invalid_argument for one outside this context's chain
    std::size_t level_of(const parms_id_type &id) const
    {
        const auto it = by_id_.find(id);
        if (it == by_id_.end()) throw std::invalid_argument("parms_id is not valid for encryption parameters");
        return it->second;
    }
    const parms_id_type &parms_id_of(std::size_t level) const
    {
        if (level < 1 || level >= levels_.size()) throw std::invalid_argument("parms_id is not valid for encryption parameters");
        return levels_[level]->parms_id();
    }
    std::size_t poly_modulus_degree() const { return hec_context_poly_degree(h_.get()); }
    std::size_t slot_count() const { return poly_modulus_degree() / 2; }
    const std::vector<std::uint64_t> &coeff_modulus() const { return moduli_; }
    std::uint32_t galois_elt_from_step(int step) const
    {
        const std::uint32_t e = hec_galois_elt_from_step(h_.get(), step);
        if (!e) check(HEC_EINVAL);
        return e;
    }
    std::vector<std::uint32_t> default_galois_elts() const
    {
        std::vector<std::uint32_t> v(hec_default_galois_elts(h_.get(), nullptr));
        hec_default_galois_elts(h_.get(), v.data());
        return v;
    }
    void set_stream(void *hip_stream) const { check(hec_context_set_stream(h_.get(), hip_stream)); }
    // multi-GPU (one process per GPU): after comm_init, BatchedMatrix::matmul diag x col shards its diagonals
    // over the ranks (hec_matmul_diag_col_sharded); every rank gets every output
    static std::vector<char> comm_unique_id()
    {
        std::vector<char> id(128);
        check(hec_comm_unique_id(id.data()));
        return id;
    }
    void comm_init(int rank, int world, const std::vector<char> &unique_id) const
    {
        check(hec_comm_init(h_.get(), rank, world, unique_id.empty() ? nullptr : unique_id.data()));
    }
    // the same sharding over the caller's own collectives (MPI, gloo, ...): hec_comm_init_ops, INTEGRATION.md §5.2
    void comm_init(int rank, int world, const hec_comm_ops &ops) const
    {
        check(hec_comm_init_ops(h_.get(), rank, world, &ops));
    }
    bool has_comm() const { return hec_context_comm(h_.get(), nullptr, nullptr) == 1; }
    void synchronize() const { check(hec_context_synchronize(h_.get())); }

private:
    std::shared_ptr<hec_context> h_;
    std::vector<std::uint64_t> moduli_;
    std::vector<std::shared_ptr<const ContextData>> levels_;  // [level], index 0 unused
    std::map<parms_id_type, std::size_t> by_id_;
};

class Ciphertext {
public:
    Ciphertext() = default;
    explicit Ciphertext(const Context &ctx) : ctx_(&ctx) { create(); }
    Ciphertext(const Ciphertext &o) : ctx_(o.ctx_)
    {
        if (o.h_) {
            create();
            check(hec_ciphertext_copy(h_, o.h_));
        }
    }
    Ciphertext(Ciphertext &&o) noexcept : ctx_(o.ctx_), h_(o.h_) { o.h_ = nullptr; }
    Ciphertext &operator=(const Ciphertext &o)
    {
        if (this == &o) return *this;
        if (!o.h_) { reset(); ctx_ = o.ctx_; return *this; }
        if (!h_ || ctx_ != o.ctx_) { reset(); ctx_ = o.ctx_; create(); }
        check(hec_ciphertext_copy(h_, o.h_));
        return *this;
    }
    Ciphertext &operator=(Ciphertext &&o) noexcept
    {
        if (this != &o) {
            reset();
            ctx_ = o.ctx_;
            h_ = o.h_;
            o.h_ = nullptr;
        }
        return *this;
    }
    ~Ciphertext() { reset(); }

    // SEAL layout host buffer u64[size][level][N] (e.g. seal::Ciphertext::data())
    void upload(const std::uint64_t *data, std::size_t size, std::size_t level, double scale)
    {
        ensure();
        check(hec_ciphertext_upload(h_, data, size, level, scale));
    }
    std::vector<std::uint64_t> download() const
    {
        std::vector<std::uint64_t> v(size() * level() * ctx_->poly_modulus_degree());
        check(hec_ciphertext_download(h_, v.data()));
        return v;
    }
    std::size_t size() const { return info().size; }
    std::size_t level() const { return info().level; }
    double scale() const { return info().scale; }
    const Context &context() const { return *ctx_; }
    // seal::Ciphertext::parms_id(): the parms_id of the ciphertext's level; coeff_modulus_size() = that level
    parms_id_type parms_id() const
    {
        if (!ctx_ || !h_) return parms_id_type{};  // SEAL's parms_id_zero for an empty ciphertext
        return ctx_->parms_id_of(level());
    }
    std::size_t coeff_modulus_size() const { return level(); }
    bool is_ntt_form() const { return true; }
    // SEAL wire format: Ciphertext::load(context, in, size) (server.cpp:120-121) returns the bytes read;
    // save(stream, compr_mode) (server.cpp:140-141; SEAL's default compression is zstd)
    std::streamoff load(const Context &ctx, const seal_byte *in, std::size_t size)
    {
        if (ctx_ != &ctx) { reset(); ctx_ = &ctx; }
        ensure();
        std::uint64_t used = 0;
        check(hec_ciphertext_load_seal(h_, in, size, &used));
        return (std::streamoff)used;
    }
    std::streamoff save(std::ostream &out, compr_mode_type mode = compr_mode_type::zstd) const
    {
        std::uint64_t w = 0;
        check(hec_ciphertext_save_seal(h_, (int)mode, nullptr, 0, &w));
        std::vector<char> b(w);
        check(hec_ciphertext_save_seal(h_, (int)mode, b.data(), w, &w));
        out.write(b.data(), (std::streamsize)w);
        return (std::streamoff)w;
    }
    hec_ciphertext *get() const { return h_; }
    // bind a default-constructed ciphertext to a context (used by out-of-place operations)
    void bind(const Context &ctx)
    {
        if (!h_ || ctx_ != &ctx) { reset(); ctx_ = &ctx; create(); }
    }

private:
    struct Info { std::size_t size, level; double scale; };
    Info info() const
    {
        if (!h_) return {0, 0, 1.0};
        std::uint64_t s = 0, l = 0;
        double sc = 0;
        check(hec_ciphertext_info(h_, &s, &l, &sc));
        return {s, l, sc};
    }
    void create()
    {
        hec_ciphertext *c = nullptr;
        check(hec_ciphertext_create(ctx_->get(), &c));
        h_ = c;
    }
    void ensure()
    {
        if (!ctx_) throw std::logic_error("ciphertext has no context");
        if (!h_) create();
    }
    void reset()
    {
        if (h_) hec_ciphertext_destroy(h_);
        h_ = nullptr;
    }
    const Context *ctx_ = nullptr;
    hec_ciphertext *h_ = nullptr;
};

class Plaintext {
public:
    Plaintext() = default;
    explicit Plaintext(const Context &ctx) : ctx_(&ctx) { create(); }
    Plaintext(const Context &ctx, const std::uint64_t *data, std::size_t level, double scale) : ctx_(&ctx)
    {
        create();
        check(hec_plaintext_upload(h_.get(), data, level, scale));
    }
    hec_plaintext *get() const { return h_.get(); }
    // bind a default-constructed plaintext to a context (CKKSEncoder::encode's destination)
    void bind(const Context &ctx)
    {
        if (!h_ || ctx_ != &ctx) { ctx_ = &ctx; create(); }
    }
    std::size_t level() const { std::uint64_t l = 0; check(hec_plaintext_info(h_.get(), &l, nullptr)); return l; }
    double scale() const { double s = 0; check(hec_plaintext_info(h_.get(), nullptr, &s)); return s; }
    parms_id_type parms_id() const { return h_ && level() ? ctx_->parms_id_of(level()) : parms_id_type{}; }
    bool is_ntt_form() const { return true; }
    // SEAL layout u64[level][N] (seal::Plaintext::data() of an NTT-form CKKS plaintext)
    std::vector<std::uint64_t> download() const
    {
        std::vector<std::uint64_t> v(level() * ctx_->poly_modulus_degree());
        check(hec_plaintext_download(h_.get(), v.data()));
        return v;
    }

private:
    void create()
    {
        hec_plaintext *p = nullptr;
        check(hec_plaintext_create(ctx_->get(), &p));
        h_.reset(p, [](hec_plaintext *x) { hec_plaintext_destroy(x); });
    }
    const Context *ctx_ = nullptr;
    std::shared_ptr<hec_plaintext> h_;
};

// seal::CKKSEncoder (reference: `CKKSEncoder cencd(ctx); cencd.encode(mat1[i], scale, pt)`,
// src/demos/matrix_operations.cpp:1106-1108) — encoding runs on the GPU (hec_encode); encode_batch
// encodes many slot vectors in one call.  Without a level the top level (all data primes) is used,
// as SEAL's first parms_id.
class CKKSEncoder {
public:
    explicit CKKSEncoder(const Context &ctx) : ctx_(&ctx) {}
    std::size_t slot_count() const { return ctx_->slot_count(); }
    void encode(const std::vector<double> &values, double scale, Plaintext &destination) const
    {
        encode(values, top(), scale, destination);
    }
    void encode(const std::vector<double> &values, std::size_t level, double scale, Plaintext &destination) const
    {
        destination.bind(*ctx_);
        hec_plaintext *p = destination.get();
        check(hec_encode(ctx_->get(), values.data(), nullptr, values.size(), 1, scale, level, &p));
    }
    void encode(const std::vector<std::complex<double>> &values, double scale, Plaintext &destination) const
    {
        encode_complex(values, top(), scale, destination);
    }
    // the parms_id overloads of SEAL (encode(values, parms_id, scale, destination)), including the scalar forms
    // he_util.h:33 and he_math.cpp:32-53 call: encode(double value, parms_id, scale, destination) puts the constant
    // round(value scale) in every coefficient (hec_encode_scalar); a complex scalar fills every slot (SEAL's
    // encode_internal(complex, ...) does the same through the vector encoder)
    void encode(const std::vector<double> &values, const parms_id_type &parms_id, double scale, Plaintext &destination) const
    {
        encode(values, ctx_->level_of(parms_id), scale, destination);
    }
    void encode(const std::vector<std::complex<double>> &values, const parms_id_type &parms_id, double scale,
                Plaintext &destination) const
    {
        encode_complex(values, ctx_->level_of(parms_id), scale, destination);
    }
    void encode(double value, const parms_id_type &parms_id, double scale, Plaintext &destination) const
    {
        const std::size_t level = ctx_->level_of(parms_id);
        destination.bind(*ctx_);
        check(hec_encode_scalar(ctx_->get(), value, scale, level, destination.get()));
    }
    void encode(double value, double scale, Plaintext &destination) const
    {
        encode(value, ctx_->first_parms_id(), scale, destination);
    }
    void encode(std::complex<double> value, const parms_id_type &parms_id, double scale, Plaintext &destination) const
    {
        encode_complex(std::vector<std::complex<double>>(slot_count(), value), ctx_->level_of(parms_id), scale,
                       destination);
    }
    // every row must have the same length (at most slot_count())
    void encode_batch(const std::vector<std::vector<double>> &rows, double scale, std::vector<Plaintext> &destination) const
    {
        const std::size_t nv = rows.empty() ? 0 : rows[0].size();
        std::vector<double> flat;
        flat.reserve(rows.size() * nv);
        for (const auto &r : rows) {
            if (r.size() != nv) throw std::invalid_argument("values has invalid size");
            flat.insert(flat.end(), r.begin(), r.end());
        }
        destination.resize(rows.size());
        std::vector<hec_plaintext *> ps(rows.size());
        for (std::size_t i = 0; i < rows.size(); ++i) { destination[i].bind(*ctx_); ps[i] = destination[i].get(); }
        check(hec_encode(ctx_->get(), flat.data(), nullptr, nv, rows.size(), scale, top(), ps.data()));
    }

private:
    std::size_t top() const { return ctx_->coeff_modulus().size() - 1; }
    void encode_complex(const std::vector<std::complex<double>> &values, std::size_t level, double scale,
                        Plaintext &destination) const
    {
        std::vector<double> re(values.size()), im(values.size());
        for (std::size_t i = 0; i < values.size(); ++i) { re[i] = values[i].real(); im[i] = values[i].imag(); }
        destination.bind(*ctx_);
        hec_plaintext *p = destination.get();
        check(hec_encode(ctx_->get(), re.data(), im.data(), values.size(), 1, scale, level, &p));
    }
    const Context *ctx_;
};

class RelinKeys {
public:
    RelinKeys() = default;
    // SEAL layout u64[L][2][K][N] (KSwitchKeys::data()[0], one PublicKey per data prime)
    RelinKeys(const Context &ctx, const std::uint64_t *data)
    {
        hec_kswitch_key *k = nullptr;
        check(hec_kswitch_key_upload(ctx.get(), data, &k));
        h_.reset(k, [](hec_kswitch_key *x) { hec_kswitch_key_destroy(x); });
    }
    hec_kswitch_key *get() const { return h_.get(); }
    // RelinKeys::load(context, in, size) (server.cpp:116)
    std::streamoff load(const Context &ctx, const seal_byte *in, std::size_t size)
    {
        hec_kswitch_key *k = nullptr;
        std::uint64_t used = 0;
        check(hec_kswitch_key_load_seal(ctx.get(), in, size, &k, &used));
        h_.reset(k, [](hec_kswitch_key *x) { hec_kswitch_key_destroy(x); });
        return (std::streamoff)used;
    }

private:
    std::shared_ptr<hec_kswitch_key> h_;
};

class GaloisKeys {
public:
    GaloisKeys() = default;
    explicit GaloisKeys(const Context &ctx)
    {
        hec_galois_keys *g = nullptr;
        check(hec_galois_keys_create(ctx.get(), &g));
        h_.reset(g, [](hec_galois_keys *x) { hec_galois_keys_destroy(x); });
    }
    void add(std::uint32_t galois_elt, const std::uint64_t *data) { check(hec_galois_keys_add(h_.get(), galois_elt, data)); }
    bool has_key(std::uint32_t galois_elt) const { return hec_galois_keys_has(h_.get(), galois_elt) != 0; }
    // GaloisKeys::load(context, in, size): every key list present in the buffer
    std::streamoff load(const Context &ctx, const seal_byte *in, std::size_t size)
    {
        if (!h_) *this = GaloisKeys(ctx);
        std::uint64_t used = 0;
        check(hec_galois_keys_load_seal(h_.get(), in, size, &used));
        return (std::streamoff)used;
    }
    hec_galois_keys *get() const { return h_.get(); }

private:
    std::shared_ptr<hec_galois_keys> h_;
};

// seal::Evaluator: const member functions, in-place and out-of-place forms
class Evaluator {
public:
    explicit Evaluator(const Context &ctx) : ctx_(&ctx) {}
    const Context &context() const { return *ctx_; }

    void negate_inplace(Ciphertext &a) const { check(hec_negate_inplace(c(), a.get())); }
    void add_inplace(Ciphertext &a, const Ciphertext &b) const { check(hec_add_inplace(c(), a.get(), b.get())); }
    void sub_inplace(Ciphertext &a, const Ciphertext &b) const { check(hec_sub_inplace(c(), a.get(), b.get())); }
    void add_plain_inplace(Ciphertext &a, const Plaintext &p) const { check(hec_add_plain_inplace(c(), a.get(), p.get())); }
    void sub_plain_inplace(Ciphertext &a, const Plaintext &p) const { check(hec_sub_plain_inplace(c(), a.get(), p.get())); }
    void multiply_inplace(Ciphertext &a, const Ciphertext &b) const { check(hec_multiply_inplace(c(), a.get(), b.get())); }
    void multiply_plain_inplace(Ciphertext &a, const Plaintext &p) const
    {
        check(hec_multiply_plain_inplace(c(), a.get(), p.get()));
    }
    void square_inplace(Ciphertext &a) const { check(hec_square_inplace(c(), a.get())); }
    void relinearize_inplace(Ciphertext &a, const RelinKeys &rk) const
    {
        check(hec_relinearize_inplace(c(), a.get(), rk.get()));
    }
    void rescale_to_next_inplace(Ciphertext &a) const { check(hec_rescale_to_next_inplace(c(), a.get())); }
    void mod_switch_to_next_inplace(Ciphertext &a) const { check(hec_mod_switch_to_next_inplace(c(), a.get())); }
    void rotate_vector_inplace(Ciphertext &a, int steps, const GaloisKeys &gk) const
    {
        check(hec_rotate_vector_inplace(c(), a.get(), steps, gk.get()));
    }
    void apply_galois_inplace(Ciphertext &a, std::uint32_t elt, const GaloisKeys &gk) const
    {
        check(hec_apply_galois_inplace(c(), a.get(), elt, gk.get()));
    }
    // Evaluator::mod_switch_to_inplace / rescale_to_inplace (encrypted, parms_id): one step at a time down the chain
    // until the ciphertext is at parms_id; SEAL's errors for an unknown parms_id and for a higher level
    void mod_switch_to_inplace(Ciphertext &a, const parms_id_type &parms_id) const
    {
        for (std::size_t n = steps_to(a, parms_id); n > 0; --n) mod_switch_to_next_inplace(a);
    }
    void rescale_to_inplace(Ciphertext &a, const parms_id_type &parms_id) const
    {
        for (std::size_t n = steps_to(a, parms_id); n > 0; --n) rescale_to_next_inplace(a);
    }

    // out-of-place forms: destination = copy, then the in-place operation (SEAL's own pattern)
    void negate(const Ciphertext &a, Ciphertext &d) const { d = a; negate_inplace(d); }
    void add(const Ciphertext &a, const Ciphertext &b, Ciphertext &d) const { d = a; add_inplace(d, b); }
    void sub(const Ciphertext &a, const Ciphertext &b, Ciphertext &d) const { d = a; sub_inplace(d, b); }
    void add_plain(const Ciphertext &a, const Plaintext &p, Ciphertext &d) const { d = a; add_plain_inplace(d, p); }
    void sub_plain(const Ciphertext &a, const Plaintext &p, Ciphertext &d) const { d = a; sub_plain_inplace(d, p); }
    void multiply(const Ciphertext &a, const Ciphertext &b, Ciphertext &d) const { d = a; multiply_inplace(d, b); }
    void multiply_plain(const Ciphertext &a, const Plaintext &p, Ciphertext &d) const
    {
        d = a;
        multiply_plain_inplace(d, p);
    }
    void square(const Ciphertext &a, Ciphertext &d) const { d = a; square_inplace(d); }
    void relinearize(const Ciphertext &a, const RelinKeys &rk, Ciphertext &d) const { d = a; relinearize_inplace(d, rk); }
    void rescale_to_next(const Ciphertext &a, Ciphertext &d) const { d = a; rescale_to_next_inplace(d); }
    void mod_switch_to_next(const Ciphertext &a, Ciphertext &d) const { d = a; mod_switch_to_next_inplace(d); }
    void rotate_vector(const Ciphertext &a, int steps, const GaloisKeys &gk, Ciphertext &d) const
    {
        d = a;
        rotate_vector_inplace(d, steps, gk);
    }
    void mod_switch_to(const Ciphertext &a, const parms_id_type &parms_id, Ciphertext &d) const
    {
        d = a;
        mod_switch_to_inplace(d, parms_id);
    }
    void rescale_to(const Ciphertext &a, const parms_id_type &parms_id, Ciphertext &d) const
    {
        d = a;
        rescale_to_inplace(d, parms_id);
    }

private:
    hec_context *c() const { return ctx_->get(); }
    std::size_t steps_to(const Ciphertext &a, const parms_id_type &parms_id) const
    {
        if (!ctx_->get_context_data(a.parms_id())) throw std::invalid_argument("encrypted is not valid for encryption parameters");
        if (!ctx_->get_context_data(parms_id)) throw std::invalid_argument("parms_id is not valid for encryption parameters");
        const std::size_t from = a.level(), to = ctx_->level_of(parms_id);
        if (from < to) throw std::invalid_argument("cannot switch to higher level modulus");
        return from - to;
    }
    const Context *ctx_;
};

}  // namespace hecdna
