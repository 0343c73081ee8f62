// SEAL 4.1 wire format for the objects the reference's socket layer moves:
// seal::Serialization::Save / Load framing (SEALHeader + members, optionally zlib- or zstd-compressed),
// Ciphertext, EncryptionParameters (CKKS), Modulus, DynArray, PublicKey and KSwitchKeys (RelinKeys,
// GaloisKeys) — what src/demos/client.cpp:113-115,238-240 writes and src/demos/server.cpp:110-122,140-152
// reads.  Host-only C++ (no device code); the C-ABI entries at the end are declared in include/hecdna.h.
//
// Layouts (SEAL 4.1 serialization.h / ciphertext.cpp / encryptionparams.cpp / kswitchkeys.cpp, restated):
//   SEALHeader (16 B): u16 magic 0xA15E, u8 header_size 0x10, u8 version_major, u8 version_minor,
//                      u8 compr_mode (0 none, 1 zlib, 2 zstd), u16 reserved, u64 size (whole object, bytes)
//   DynArray<u64>:     header, u64 count, count words
//   Ciphertext:        header, parms_id (4 x u64), u8 is_ntt_form, u64 size, u64 poly_modulus_degree,
//                      u64 coeff_modulus_size, f64 scale, u64 correction_factor (4.x), DynArray data
//                      (seeded: data holds c0 only and a UniformRandomGeneratorInfo follows)
//   Modulus:           header, u64 value
//   EncryptionParameters: header, u8 scheme (ckks = 2), u64 N, u64 count, count x Modulus, Modulus plain
//   PublicKey:         header, Ciphertext
//   KSwitchKeys:       header, parms_id, u64 dim1, dim1 x (u64 dim2, dim2 x PublicKey)
//   parms_id:          BLAKE2b-256 of the u64 words {scheme, N, q_0..q_{k-1}, plain modulus}
//                      (EncryptionParameters::compute_parms_id; the plain modulus of CKKS is one zero word)
// Parity status: no SEAL-written bytes exist under /root/reference and SEAL cannot run here, so this is
// pinned by structure tests and round trips only.
#include <dlfcn.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "hecdna.h"

namespace {
using u64 = uint64_t;
using u8 = uint8_t;

thread_local std::string g_io_err;

// ------------------------------------------------------------------ BLAKE2b (RFC 7693)
const u64 kIV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL, 0xa54ff53a5f1d36f1ULL,
                    0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL, 0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
const u8 kSigma[12][16] = {{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
                           {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
                           {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
                           {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
                           {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
                           {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
                           {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
                           {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
                           {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
                           {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
                           {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
                           {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
inline u64 rotr(u64 x, int n) { return (x >> n) | (x << (64 - n)); }

void blake2b_compress(u64 h[8], const u8 block[128], u64 t, bool last)
{
    u64 m[16], v[16];
    for (int i = 0; i < 16; ++i) std::memcpy(&m[i], block + 8 * i, 8);  // little-endian host
    for (int i = 0; i < 8; ++i) { v[i] = h[i]; v[i + 8] = kIV[i]; }
    v[12] ^= t;  // byte counter (messages here are far below 2^64 bytes)
    if (last) v[14] = ~v[14];
    auto G = [&](int a, int b, int c, int d, u64 x, u64 y) {
        v[a] = v[a] + v[b] + x; v[d] = rotr(v[d] ^ v[a], 32);
        v[c] = v[c] + v[d];     v[b] = rotr(v[b] ^ v[c], 24);
        v[a] = v[a] + v[b] + y; v[d] = rotr(v[d] ^ v[a], 16);
        v[c] = v[c] + v[d];     v[b] = rotr(v[b] ^ v[c], 63);
    };
    for (int r = 0; r < 12; ++r) {
        const u8 *s = kSigma[r];
        G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

// BLAKE2b over an explicit 64-byte parameter block (RFC 7693 §2.5; BLAKE2 paper §2.8), keyed when keylen > 0:
// the key, zero-padded to one 128-byte block, is hashed ahead of the input.
void blake2b_param(u8 *out, std::size_t outlen, const u8 *in, std::size_t inlen, const u8 *key, std::size_t keylen,
                   const u8 param[64])
{
    u64 h[8];
    for (int i = 0; i < 8; ++i) {
        u64 w;
        std::memcpy(&w, param + 8 * i, 8);
        h[i] = kIV[i] ^ w;
    }
    std::vector<u8> msg;
    if (keylen) {
        msg.assign(128, 0);
        std::memcpy(msg.data(), key, keylen);
        msg.insert(msg.end(), in, in + inlen);
        in = msg.data();
        inlen = msg.size();
    }
    u8 block[128];
    u64 t = 0;
    while (inlen > 128) {
        t += 128;
        blake2b_compress(h, in, t, false);
        in += 128;
        inlen -= 128;
    }
    std::memset(block, 0, 128);
    if (inlen) std::memcpy(block, in, inlen);
    t += inlen;
    blake2b_compress(h, block, t, true);
    u8 full[64];
    std::memcpy(full, h, 64);
    std::memcpy(out, full, outlen);
}

// unkeyed sequential BLAKE2b with an outlen-byte digest (util::HashFunction behind parms_id)
void blake2b(u8 *out, std::size_t outlen, const u8 *in, std::size_t inlen)
{
    u8 param[64] = {};
    param[0] = (u8)outlen;
    param[2] = 1;  // fanout
    param[3] = 1;  // depth
    blake2b_param(out, outlen, in, inlen, nullptr, 0, param);
}

// BLAKE2Xb (the BLAKE2X note; reference blake2xb.c, which SEAL 4.1 vendors as util/blake2xb.c): a keyed
// root hash whose parameter block carries the XOF length, then ceil(outlen / 64) unkeyed leaf hashes of the
// root, leaf i with node_offset i and digest length min(64, remaining).
void blake2xb(u8 *out, std::size_t outlen, const u8 *in, std::size_t inlen, const u8 *key, std::size_t keylen)
{
    u8 param[64] = {};
    param[0] = 64;
    param[1] = (u8)keylen;
    param[2] = 1;
    param[3] = 1;
    const uint32_t xof = (uint32_t)outlen;
    std::memcpy(param + 12, &xof, 4);
    u8 root[64];
    blake2b_param(root, 64, in, inlen, key, keylen, param);
    param[1] = 0;     // key_length
    param[2] = 0;     // fanout
    param[3] = 0;     // depth
    param[4] = 64;    // leaf_length (u32 LE)
    param[17] = 64;   // inner_length
    for (uint32_t i = 0; outlen > 0; ++i) {
        const std::size_t bs = outlen < 64 ? outlen : 64;
        param[0] = (u8)bs;
        std::memcpy(param + 8, &i, 4);  // node_offset
        blake2b_param(out, bs, root, 64, nullptr, 0, param);
        out += bs;
        outlen -= bs;
    }
}

// SHAKE256 (FIPS 202: Keccak-f[1600], rate 136 bytes, domain byte 0x1F), behind SEAL's Shake256PRNG.
void keccak_f1600(u64 a[25])
{
    static const u64 rc[24] = {
        0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL, 0x8000000080008000ULL,
        0x000000000000808bULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
        0x000000000000008aULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
        0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
        0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800aULL, 0x800000008000000aULL,
        0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
    static const int rho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    auto rotl = [](u64 x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; };
    for (int r = 0; r < 24; ++r) {
        u64 c[5], b[25];
        for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        for (int x = 0; x < 5; ++x) {
            const u64 d = c[(x + 4) % 5] ^ rotl(c[(x + 1) % 5], 1);
            for (int y = 0; y < 25; y += 5) a[y + x] ^= d;
        }
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl(a[x + 5 * y], rho[x + 5 * y]);
        for (int y = 0; y < 25; y += 5)
            for (int x = 0; x < 5; ++x) a[y + x] = b[y + x] ^ (~b[y + (x + 1) % 5] & b[y + (x + 2) % 5]);
        a[0] ^= rc[r];
    }
}
void shake256(u8 *out, std::size_t outlen, const u8 *in, std::size_t inlen)
{
    constexpr std::size_t rate = 136;
    u64 a[25] = {};
    auto absorb = [&](const u8 *blk) {
        for (std::size_t i = 0; i < rate / 8; ++i) {
            u64 w;
            std::memcpy(&w, blk + 8 * i, 8);
            a[i] ^= w;
        }
        keccak_f1600(a);
    };
    for (; inlen >= rate; in += rate, inlen -= rate) absorb(in);
    u8 last[rate] = {};
    if (inlen) std::memcpy(last, in, inlen);
    last[inlen] ^= 0x1F;
    last[rate - 1] ^= 0x80;
    absorb(last);
    while (outlen) {
        const std::size_t k = std::min(outlen, rate);
        std::memcpy(out, a, k);  // little-endian lanes
        out += k;
        outlen -= k;
        if (outlen) keccak_f1600(a);
    }
}

// SEAL 4.1 UniformRandomGenerator (randomgen.cpp): a byte stream of 4096-byte buffers served in order by
// generate(); buffer k is Blake2xbPRNG's BLAKE2Xb(input = the u64 counter k, key = the 64-byte
// prng_seed_type) or Shake256PRNG's SHAKE256(seed || u64 counter k).
struct PrngStream {
    int type = 1;  // prng_type: 1 blake2xb, 2 shake256
    u8 seed[64];
    u64 counter = 0;
    u8 buf[4096];
    std::size_t head = sizeof(buf);
    void refill()
    {
        if (type == 1) {
            blake2xb(buf, sizeof(buf), reinterpret_cast<const u8 *>(&counter), 8, seed, 64);
        } else {
            u8 ext[72];
            std::memcpy(ext, seed, 64);
            std::memcpy(ext + 64, &counter, 8);
            shake256(buf, sizeof(buf), ext, sizeof(ext));
        }
        ++counter;
        head = 0;
    }
    void generate(u8 *dst, std::size_t n)
    {
        while (n) {
            if (head == sizeof(buf)) refill();
            const std::size_t k = std::min(n, sizeof(buf) - head);
            std::memcpy(dst, buf + head, k);
            head += k;
            dst += k;
            n -= k;
        }
    }
};

// SEAL 4.1 sample_poly_uniform (util/rlwe.cpp), which Ciphertext::expand_seed runs into c1 for a version-4
// object: fill the level x N words from the stream in one draw, then per prime q_j reject each word
// >= max_multiple = (2^64 - 1) - ((2^64 - 1) mod q_j) - 1 by redrawing it from the stream's continuation,
// and reduce mod q_j.  In NTT form (CKKS) the uniform c1 is used as drawn.
void sample_poly_uniform(PrngStream &prng, const u64 *q, u64 level, u64 N, u64 *dst)
{
    prng.generate(reinterpret_cast<u8 *>(dst), level * N * 8);
    const u64 max_random = ~0ULL;
    for (u64 j = 0; j < level; ++j, dst += N) {
        const u64 max_multiple = max_random - max_random % q[j] - 1;
        for (u64 i = 0; i < N; ++i) {
            u64 v = dst[i];
            while (v >= max_multiple) prng.generate(reinterpret_cast<u8 *>(&v), 8);
            dst[i] = v % q[j];
        }
    }
}

// ------------------------------------------------------------------ framing
constexpr uint16_t kMagic = 0xA15E;
constexpr u8 kHeaderSize = 0x10;
constexpr u8 kVersionMajor = 4, kVersionMinor = 1;

struct Header {
    uint16_t magic = kMagic;
    u8 header_size = kHeaderSize, major = kVersionMajor, minor = kVersionMinor, compr = 0;
    uint16_t reserved = 0;
    u64 size = 0;
};
static_assert(sizeof(Header) == 16, "SEALHeader is 16 bytes");

struct Reader {
    const u8 *p, *end;
    void need(std::size_t n) const
    {
        if ((std::size_t)(end - p) < n) throw std::invalid_argument("SEAL object is truncated");
    }
    template <class T>
    T get()
    {
        need(sizeof(T));
        T v;
        std::memcpy(&v, p, sizeof(T));
        p += sizeof(T);
        return v;
    }
    void bytes(void *dst, std::size_t n)
    {
        need(n);
        std::memcpy(dst, p, n);
        p += n;
    }
};
struct Writer {
    std::vector<u8> b;
    template <class T>
    void put(const T &v)
    {
        const u8 *s = reinterpret_cast<const u8 *>(&v);
        b.insert(b.end(), s, s + sizeof(T));
    }
    void bytes(const void *s, std::size_t n)
    {
        const u8 *c = static_cast<const u8 *>(s);
        b.insert(b.end(), c, c + n);
    }
};

// ---- compression (libz / libzstd loaded on first use)
struct Zstd {
    void *(*create_d)() = nullptr;
    std::size_t (*free_d)(void *) = nullptr;
    std::size_t (*init_d)(void *) = nullptr;
    std::size_t (*decompress_stream)(void *, void *, void *) = nullptr;
    std::size_t (*compress)(void *, std::size_t, const void *, std::size_t, int) = nullptr;
    std::size_t (*bound)(std::size_t) = nullptr;
    unsigned (*is_error)(std::size_t) = nullptr;
};
struct ZInBuf { const void *src; std::size_t size, pos; };
struct ZOutBuf { void *dst; std::size_t size, pos; };
const Zstd &zstd()
{
    static Zstd z;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        z.create_d = (decltype(z.create_d))dlsym(h, "ZSTD_createDStream");
        z.free_d = (decltype(z.free_d))dlsym(h, "ZSTD_freeDStream");
        z.init_d = (decltype(z.init_d))dlsym(h, "ZSTD_initDStream");
        z.decompress_stream = (decltype(z.decompress_stream))dlsym(h, "ZSTD_decompressStream");
        z.compress = (decltype(z.compress))dlsym(h, "ZSTD_compress");
        z.bound = (decltype(z.bound))dlsym(h, "ZSTD_compressBound");
        z.is_error = (decltype(z.is_error))dlsym(h, "ZSTD_isError");
    });
    if (!z.create_d || !z.decompress_stream || !z.compress || !z.bound || !z.is_error)
        throw std::logic_error("zstd (libzstd.so.1) is not available");
    return z;
}
struct Zlib {
    int (*inflate_init2)(z_streamp, int, const char *, int) = nullptr;
    int (*inflate)(z_streamp, int) = nullptr;
    int (*inflate_end)(z_streamp) = nullptr;
    int (*compress2)(Bytef *, uLongf *, const Bytef *, uLong, int) = nullptr;
    uLong (*bound)(uLong) = nullptr;
};
const Zlib &zlib()
{
    static Zlib z;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("libz.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        z.inflate_init2 = (decltype(z.inflate_init2))dlsym(h, "inflateInit2_");
        z.inflate = (decltype(z.inflate))dlsym(h, "inflate");
        z.inflate_end = (decltype(z.inflate_end))dlsym(h, "inflateEnd");
        z.compress2 = (decltype(z.compress2))dlsym(h, "compress2");
        z.bound = (decltype(z.bound))dlsym(h, "compressBound");
    });
    if (!z.inflate_init2 || !z.inflate || !z.compress2) throw std::logic_error("zlib (libz.so.1) is not available");
    return z;
}

// Decompressed member bytes are bounded: a client's bytes arrive over the socket (server.cpp:110-122), so a small
// compressed payload must not expand without limit.  kMaxCtObject covers a ciphertext object (size <= 16 polys,
// N <= 2^17, <= 64 limbs of u64: 1 GiB of words).  A KSwitchKeys object is bounded by its caller: the device
// loaders know N, K and L and pass the size of the key lists they accept (hec_engine.hip); the context-free
// entry points use keys_default_limit(): kMaxKeysObjectDefault (16 GiB: SEAL's default GaloisKeys take 1.67 GB at
// N = 2^15, L = 10 and 8.84 GB at the cfg5 size N = 2^16, L = 16, 31 lists) bounded by half the host's available
// memory (the object is inflated in host memory), at least 1 GiB; the *_ex forms take an explicit limit.  The output buffer doubles from a small start, so a rejected payload has
// cost at most twice the limit.
constexpr std::size_t kMaxCtObject = (std::size_t)1 << 31;
constexpr std::size_t kMaxKeysObjectDefault = (std::size_t)1 << 34;
std::size_t keys_default_limit()
{
    const long pages = sysconf(_SC_AVPHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
    std::size_t lim = kMaxKeysObjectDefault;
    if (pages > 0 && psz > 0) lim = std::min(lim, (std::size_t)pages * (std::size_t)psz / 2);
    return std::max(lim, (std::size_t)1 << 30);
}
void check_growth(std::size_t want, std::size_t max_out)
{
    if (want > max_out) throw std::invalid_argument("decompressed SEAL object exceeds the size limit");
}

std::vector<u8> inflate_zlib(const u8 *src, std::size_t n, std::size_t max_out)
{
    const Zlib &z = zlib();
    for (int wbits : {15 + 32, -15}) {  // zlib / gzip framing, then a raw deflate stream
        z_stream s{};
        if (z.inflate_init2(&s, wbits, ZLIB_VERSION, (int)sizeof(z_stream)) != Z_OK) continue;
        std::vector<u8> out(std::min(std::max<std::size_t>(4 * n, 4096), max_out + 1));
        s.next_in = const_cast<Bytef *>(src);
        s.avail_in = (uInt)n;
        int rc = Z_OK;
        while (rc == Z_OK) {
            if (s.total_out == out.size()) {
                if (s.total_out > max_out) {
                    z.inflate_end(&s);  // the stream state is released before the rejection
                    check_growth(s.total_out, max_out);
                }
                out.resize(std::min(2 * out.size(), max_out + 1));
            }
            s.next_out = out.data() + s.total_out;
            s.avail_out = (uInt)(out.size() - s.total_out);
            rc = z.inflate(&s, Z_NO_FLUSH);
            if (rc == Z_BUF_ERROR && s.avail_out == 0) rc = Z_OK;
        }
        const std::size_t got = s.total_out;
        z.inflate_end(&s);
        if (rc == Z_STREAM_END) {
            check_growth(got, max_out);
            out.resize(got);
            return out;
        }
    }
    throw std::invalid_argument("zlib payload of the SEAL object is corrupt");
}
std::vector<u8> inflate_zstd(const u8 *src, std::size_t n, std::size_t max_out)
{
    const Zstd &z = zstd();
    void *ds = z.create_d();
    z.init_d(ds);
    std::vector<u8> out(std::min(std::max<std::size_t>(4 * n, 4096), max_out + 1));
    ZInBuf in{src, n, 0};
    ZOutBuf ob{out.data(), out.size(), 0};
    std::size_t rc = 1;
    while (in.pos < in.size || rc != 0) {
        if (ob.pos == ob.size) {
            if (ob.pos > max_out) {
                z.free_d(ds);
                check_growth(ob.pos, max_out);
            }
            out.resize(std::min(2 * out.size(), max_out + 1));
            ob.dst = out.data();
            ob.size = out.size();
        }
        const std::size_t before_in = in.pos, before_out = ob.pos;
        rc = z.decompress_stream(ds, &ob, &in);
        if (z.is_error(rc)) { z.free_d(ds); throw std::invalid_argument("zstd payload of the SEAL object is corrupt"); }
        if (rc == 0 && in.pos == in.size) break;
        if (in.pos == before_in && ob.pos == before_out && ob.pos < ob.size) {
            z.free_d(ds);
            throw std::invalid_argument("zstd payload of the SEAL object is truncated");
        }
    }
    z.free_d(ds);
    check_growth(ob.pos, max_out);
    out.resize(ob.pos);
    return out;
}

// One SEAL object: its header, then the members (decompressed when needed, at most max_out bytes).  Returns the
// member bytes and advances r past the whole object.
// Decompression budget of the object being loaded: every compressed payload nested in it (a KSwitchKeys object's
// PublicKeys, their DynArrays) draws from it, so nested compressed members cannot multiply the caller's limit.
thread_local std::size_t t_inflate_budget = SIZE_MAX;
struct InflateBudget {
    std::size_t saved;
    explicit InflateBudget(std::size_t b) : saved(t_inflate_budget) { t_inflate_budget = b; }
    ~InflateBudget() { t_inflate_budget = saved; }
};

std::vector<u8> open_object(Reader &r, std::size_t max_out = kMaxCtObject)
{
    const Header h = r.get<Header>();
    if (h.magic != kMagic || h.header_size != kHeaderSize) throw std::invalid_argument("loaded SEALHeader is invalid");
    if (h.major != 3 && h.major != 4) throw std::invalid_argument("loaded SEALHeader version is not supported");
    if (h.size < sizeof(Header)) throw std::invalid_argument("loaded SEALHeader is invalid");
    const std::size_t n = h.size - sizeof(Header);
    r.need(n);
    const u8 *payload = r.p;
    r.p += n;
    if (h.compr == 0) return std::vector<u8>(payload, payload + n);
    if (h.compr != 1 && h.compr != 2) throw std::invalid_argument("unsupported compression mode");
    std::vector<u8> out = h.compr == 1 ? inflate_zlib(payload, n, std::min(max_out, t_inflate_budget))
                                       : inflate_zstd(payload, n, std::min(max_out, t_inflate_budget));
    if (t_inflate_budget != SIZE_MAX) t_inflate_budget -= out.size();
    return out;
}
// wrap members into a SEAL object with the given compression
void close_object(Writer &w, const std::vector<u8> &members, int compr)
{
    std::vector<u8> body;
    if (compr == 0) body = members;
    else if (compr == 2) {
        const Zstd &z = zstd();
        body.resize(z.bound(members.size()));
        const std::size_t k = z.compress(body.data(), body.size(), members.data(), members.size(), 3);
        if (z.is_error(k)) throw std::logic_error("zstd compression failed");
        body.resize(k);
    } else if (compr == 1) {
        const Zlib &z = zlib();
        uLongf k = z.bound ? z.bound((uLong)members.size()) : (uLongf)(members.size() + members.size() / 100 + 64);
        body.resize(k);
        if (z.compress2(body.data(), &k, members.data(), (uLong)members.size(), Z_DEFAULT_COMPRESSION) != Z_OK)
            throw std::logic_error("zlib compression failed");
        body.resize(k);
    } else {
        throw std::invalid_argument("unsupported compression mode");
    }
    Header h;
    h.compr = (u8)compr;
    h.size = sizeof(Header) + body.size();
    w.put(h);
    w.bytes(body.data(), body.size());
}

// ---- objects
struct CtData {
    u64 parms_id[4] = {0, 0, 0, 0};
    bool ntt = true;
    u64 size = 0, N = 0, level = 0, correction = 1;
    double scale = 1.0;
    std::vector<u64> data;  // u64[size][level][N]
    bool seeded = false;
    int major = 4;
    u8 prng_type = 0;  // UniformRandomGeneratorInfo of a seeded ciphertext: 1 blake2xb, 2 shake256
    u8 seed[64] = {};
};

CtData parse_ciphertext(Reader &outer, int major)
{
    std::vector<u8> m = open_object(outer);
    Reader r{m.data(), m.data() + m.size()};
    CtData c;
    r.bytes(c.parms_id, 32);
    c.ntt = r.get<u8>() != 0;
    c.size = r.get<u64>();
    c.N = r.get<u64>();
    c.level = r.get<u64>();
    c.scale = r.get<double>();
    if (major >= 4) c.correction = r.get<u64>();
    if (c.size > 16 || c.N > (1u << 17) || c.level > 64) throw std::invalid_argument("ciphertext data is invalid");
    std::vector<u8> dm = open_object(r);  // DynArray<u64>
    Reader d{dm.data(), dm.data() + dm.size()};
    const u64 count = d.get<u64>();
    const u64 full = c.size * c.N * c.level;
    if (count != full && !(c.size == 2 && count == c.N * c.level)) throw std::invalid_argument("ciphertext data is invalid");
    d.need(count * 8);  // before allocating: the payload must hold the words it announces
    c.data.resize(count);
    d.bytes(c.data.data(), count * 8);
    c.major = major;
    if (count != full) {  // c0 only + UniformRandomGeneratorInfo (u8 prng_type, 8 x u64 seed): expand_seed
        c.seeded = true;
        std::vector<u8> im = open_object(r);
        Reader ir{im.data(), im.data() + im.size()};
        c.prng_type = ir.get<u8>();
        ir.bytes(c.seed, 64);
    }
    return c;
}
void emit_ciphertext(Writer &w, const CtData &c, int compr)
{
    Writer m;
    m.bytes(c.parms_id, 32);
    m.put((u8)(c.ntt ? 1 : 0));
    m.put(c.size);
    m.put(c.N);
    m.put(c.level);
    m.put(c.scale);
    m.put(c.correction);
    Writer d;
    d.put((u64)c.data.size());
    d.bytes(c.data.data(), c.data.size() * 8);
    close_object(m, d.b, 0);
    close_object(w, m.b, compr);
}

void parms_id_of(u64 N, const u64 *moduli, u64 count, u64 out[4])
{
    std::vector<u64> words;
    words.push_back(2);  // scheme_type::ckks
    words.push_back(N);
    for (u64 i = 0; i < count; ++i) words.push_back(moduli[i]);
    words.push_back(0);  // plain_modulus (zero for CKKS)
    blake2b(reinterpret_cast<u8 *>(out), 32, reinterpret_cast<const u8 *>(words.data()), words.size() * 8);
}

// Ciphertext::expand_seed (ciphertext.cpp) for a version-4 object: c1 = sample_poly_uniform over the
// ciphertext's own primes q_0..q_{level-1}, drawn from the seed's PRNG (Blake2xbPRNG, SEAL's default, or
// Shake256PRNG).
void expand_seed(CtData &c, const u64 *q, u64 count)
{
    if (!q) throw std::invalid_argument("seeded ciphertext: the context's coeff_modulus is needed to expand it");
    if (count < c.level) throw std::invalid_argument("ciphertext data is invalid");
    u64 want[4];
    parms_id_of(c.N, q, c.level, want);
    if (std::memcmp(want, c.parms_id, 32) != 0) throw std::invalid_argument("ciphertext data is invalid");
    if (c.major != 4) throw std::invalid_argument("seeded ciphertext: only SEAL 4.x seed expansion is supported");
    if (c.prng_type != 1 && c.prng_type != 2)
        throw std::invalid_argument("seeded ciphertext: unsupported prng_type");
    const u64 half = c.N * c.level;
    c.data.resize(2 * half);
    PrngStream prng;
    prng.type = c.prng_type;
    std::memcpy(prng.seed, c.seed, 64);
    sample_poly_uniform(prng, q, c.level, c.N, c.data.data() + half);
    c.seeded = false;
}

// a status chosen by a caller's callback (hec_seal_kswitch_keys_foreach's visit), returned unchanged by io_guard
struct CallerStatus : std::runtime_error {
    int rc;
    explicit CallerStatus(int r) : std::runtime_error("key list rejected by the caller"), rc(r) {}
};

template <class F>
int io_guard(F &&f)
{
    try {
        f();
        return HEC_OK;
    } catch (const CallerStatus &e) {
        g_io_err = e.what();
        return e.rc;
    } catch (const std::invalid_argument &e) {
        g_io_err = e.what();
        return HEC_EINVAL;
    } catch (const std::exception &e) {
        g_io_err = e.what();
        return HEC_ELOGIC;
    }
}
void copy_out(const std::vector<u8> &b, void *out, uint64_t cap, uint64_t *written)
{
    if (written) *written = b.size();
    if (!out) return;
    if (cap < b.size()) throw std::invalid_argument("output buffer is too small");
    std::memcpy(out, b.data(), b.size());
}
// KSwitchKeys (RelinKeys / GaloisKeys) in one pass: the object is opened and decompressed once, and every
// non-empty key list (its PublicKeys' data back to back, the engine's key layout u64[L][2][K][N]) is handed to
// visit(index, words, nwords) as soon as it is parsed.  SEAL's GaloisKeys carry N key lists, almost all empty
// (KeyGenerator::create_galois_keys resizes the list array to the ring degree), so a per-list reparse would cost
// N full parses.
template <class F>
void walk_kswitch_keys(const void *bytes, uint64_t nbytes, uint64_t max_bytes, uint64_t *lists, uint64_t *consumed,
                       F &&visit)
{
    if (!bytes) throw std::invalid_argument("invalid argument");
    Reader outer{static_cast<const u8 *>(bytes), static_cast<const u8 *>(bytes) + nbytes};
    Header h;
    std::memcpy(&h, bytes, std::min<uint64_t>(nbytes, sizeof(h)));
    InflateBudget budget(max_bytes ? (std::size_t)max_bytes : keys_default_limit());
    std::vector<u8> m = open_object(outer, t_inflate_budget);
    Reader r{m.data(), m.data() + m.size()};
    u64 pid[4];
    r.bytes(pid, 32);
    const u64 dim1 = r.get<u64>();
    if (lists) *lists = dim1;
    std::vector<u64> got;
    for (u64 i = 0; i < dim1; ++i) {
        const u64 dim2 = r.get<u64>();
        got.clear();
        for (u64 j = 0; j < dim2; ++j) {
            std::vector<u8> pk = open_object(r, kMaxCtObject);  // PublicKey
            Reader rp{pk.data(), pk.data() + pk.size()};
            const CtData c = parse_ciphertext(rp, h.major);
            got.insert(got.end(), c.data.begin(), c.data.end());
        }
        if (dim2) visit(i, got);
    }
    if (consumed) *consumed = (uint64_t)(outer.p - static_cast<const u8 *>(bytes));
}

}  // namespace

extern "C" {

const char *hec_seal_last_error(void) { return g_io_err.c_str(); }
uint64_t hec_seal_kswitch_keys_default_limit(void) { return keys_default_limit(); }

int hec_seal_blake2b(const void *in, uint64_t n, uint64_t outlen, void *out)
{
    return io_guard([&] {
        if (!out || outlen < 1 || outlen > 64 || (!in && n)) throw std::invalid_argument("invalid argument");
        blake2b(static_cast<u8 *>(out), outlen, static_cast<const u8 *>(in), n);
    });
}

int hec_seal_parms_id(uint64_t N, const uint64_t *coeff_modulus, uint64_t count, uint64_t out[4])
{
    return io_guard([&] {
        if (!coeff_modulus || !out || !count) throw std::invalid_argument("invalid argument");
        parms_id_of(N, coeff_modulus, count, out);
    });
}

int hec_seal_ciphertext_load_ex(const void *bytes, uint64_t nbytes, const uint64_t *coeff_modulus, uint64_t count,
                                uint64_t *size, uint64_t *level, uint64_t *N, double *scale, uint64_t parms_id[4],
                                uint64_t *data, uint64_t data_words, uint64_t *consumed)
{
    return io_guard([&] {
        if (!bytes) throw std::invalid_argument("invalid argument");
        Reader r{static_cast<const u8 *>(bytes), static_cast<const u8 *>(bytes) + nbytes};
        Header h;
        std::memcpy(&h, bytes, std::min<uint64_t>(nbytes, sizeof(h)));
        CtData c = parse_ciphertext(r, h.major);
        if (c.seeded) {
            if (!coeff_modulus)
                throw std::invalid_argument("seeded ciphertext: load it with hec_seal_ciphertext_load_ex and the "
                                            "context's coeff_modulus (Ciphertext::expand_seed)");
            // the expansion is only paid for when the caller asks for the words
            if (data) expand_seed(c, coeff_modulus, count);
            else if (count < c.level) throw std::invalid_argument("ciphertext data is invalid");
        }
        if (!c.ntt) throw std::invalid_argument("CKKS ciphertext is not in NTT form");
        if (size) *size = c.size;
        if (level) *level = c.level;
        if (N) *N = c.N;
        if (scale) *scale = c.scale;
        if (parms_id) std::memcpy(parms_id, c.parms_id, 32);
        if (consumed) *consumed = (uint64_t)(r.p - static_cast<const u8 *>(bytes));
        if (data) {
            if (data_words < c.data.size()) throw std::invalid_argument("output buffer is too small");
            std::memcpy(data, c.data.data(), c.data.size() * 8);
        }
    });
}

int hec_seal_ciphertext_load(const void *bytes, uint64_t nbytes, uint64_t *size, uint64_t *level, uint64_t *N,
                             double *scale, uint64_t parms_id[4], uint64_t *data, uint64_t data_words,
                             uint64_t *consumed)
{
    return hec_seal_ciphertext_load_ex(bytes, nbytes, nullptr, 0, size, level, N, scale, parms_id, data, data_words,
                                       consumed);
}

int hec_seal_shake256(const void *in, uint64_t n, uint64_t outlen, void *out)
{
    return io_guard([&] {
        if (!out || !outlen || (!in && n)) throw std::invalid_argument("invalid argument");
        shake256(static_cast<u8 *>(out), outlen, static_cast<const u8 *>(in), n);
    });
}

int hec_seal_blake2xb(const void *in, uint64_t n, const void *key, uint64_t keylen, uint64_t outlen, void *out)
{
    return io_guard([&] {
        if (!out || outlen < 1 || outlen > 0xFFFFFFFFull || keylen > 64 || (!in && n) || (!key && keylen))
            throw std::invalid_argument("invalid argument");
        blake2xb(static_cast<u8 *>(out), outlen, static_cast<const u8 *>(in), n, static_cast<const u8 *>(key), keylen);
    });
}

int hec_seal_ciphertext_save(const uint64_t *data, uint64_t size, uint64_t level, uint64_t N, double scale,
                             const uint64_t *coeff_modulus, int compr_mode, void *out, uint64_t cap, uint64_t *written)
{
    return io_guard([&] {
        if (!data || !coeff_modulus || !size || !level || !N) throw std::invalid_argument("invalid argument");
        CtData c;
        parms_id_of(N, coeff_modulus, level, c.parms_id);  // the parms_id of the ciphertext's level
        c.size = size;
        c.level = level;
        c.N = N;
        c.scale = scale;
        c.data.assign(data, data + size * level * N);
        Writer w;
        emit_ciphertext(w, c, compr_mode);
        copy_out(w.b, out, cap, written);
    });
}

int hec_seal_parms_load(const void *bytes, uint64_t nbytes, uint64_t *N, uint64_t *coeff_modulus, uint64_t cap,
                        uint64_t *count, uint64_t *consumed)
{
    return io_guard([&] {
        if (!bytes || !count) throw std::invalid_argument("invalid argument");
        Reader outer{static_cast<const u8 *>(bytes), static_cast<const u8 *>(bytes) + nbytes};
        std::vector<u8> m = open_object(outer);
        Reader r{m.data(), m.data() + m.size()};
        const u8 scheme = r.get<u8>();
        if (scheme != 2) throw std::invalid_argument("scheme is not CKKS");
        const u64 n = r.get<u64>(), k = r.get<u64>();
        if (k > 64) throw std::invalid_argument("coeff_modulus is invalid");
        std::vector<u64> q(k);
        for (u64 i = 0; i < k; ++i) {
            std::vector<u8> mm = open_object(r);
            Reader rm{mm.data(), mm.data() + mm.size()};
            q[i] = rm.get<u64>();
        }
        (void)open_object(r);  // plain_modulus (unused by CKKS)
        if (N) *N = n;
        *count = k;
        if (coeff_modulus) {
            if (cap < k) throw std::invalid_argument("output buffer is too small");
            std::memcpy(coeff_modulus, q.data(), k * 8);
        }
        if (consumed) *consumed = (uint64_t)(outer.p - static_cast<const u8 *>(bytes));
    });
}

int hec_seal_parms_save(uint64_t N, const uint64_t *coeff_modulus, uint64_t count, int compr_mode, void *out,
                        uint64_t cap, uint64_t *written)
{
    return io_guard([&] {
        if (!coeff_modulus || !count) throw std::invalid_argument("invalid argument");
        Writer m;
        m.put((u8)2);
        m.put((u64)N);
        m.put((u64)count);
        for (u64 i = 0; i < count; ++i) {
            Writer q;
            q.put(coeff_modulus[i]);
            close_object(m, q.b, 0);
        }
        Writer pm;
        pm.put((u64)0);
        close_object(m, pm.b, 0);
        Writer w;
        close_object(w, m.b, compr_mode);
        copy_out(w.b, out, cap, written);
    });
}

// KSwitchKeys key list `index` (RelinKeys: 0; GaloisKeys: (galois_elt - 1) / 2) as the engine's key layout
// u64[L][2][K][N].  With index = UINT64_MAX only *lists (dim1) is reported; *words = the list's word count (0 when
// that list is empty).
int hec_seal_kswitch_keys_load_ex(const void *bytes, uint64_t nbytes, uint64_t index, uint64_t max_bytes,
                                  uint64_t *lists, uint64_t *out, uint64_t cap_words, uint64_t *words,
                                  uint64_t *consumed)
{
    return io_guard([&] {
        std::vector<u64> got;
        walk_kswitch_keys(bytes, nbytes, max_bytes, lists, consumed, [&](u64 i, const std::vector<u64> &w) {
            if (i == index) got = w;
        });
        if (words) *words = got.size();
        if (out && index != UINT64_MAX) {
            if (cap_words < got.size()) throw std::invalid_argument("output buffer is too small");
            std::memcpy(out, got.data(), got.size() * 8);
        }
    });
}

int hec_seal_kswitch_keys_load(const void *bytes, uint64_t nbytes, uint64_t index, uint64_t *lists, uint64_t *out,
                               uint64_t cap_words, uint64_t *words, uint64_t *consumed)
{
    return hec_seal_kswitch_keys_load_ex(bytes, nbytes, index, 0, lists, out, cap_words, words, consumed);
}

int hec_seal_kswitch_keys_foreach_ex(const void *bytes, uint64_t nbytes, uint64_t max_bytes,
                                     int (*visit)(void *user, uint64_t index, const uint64_t *words, uint64_t nwords),
                                     void *user, uint64_t *lists, uint64_t *consumed)
{
    return io_guard([&] {
        if (!visit) throw std::invalid_argument("invalid argument");
        walk_kswitch_keys(bytes, nbytes, max_bytes, lists, consumed, [&](u64 i, const std::vector<u64> &w) {
            const int rc = visit(user, i, w.data(), w.size());
            if (rc != HEC_OK) throw CallerStatus(rc);
        });
    });
}

int hec_seal_kswitch_keys_foreach(const void *bytes, uint64_t nbytes,
                                  int (*visit)(void *user, uint64_t index, const uint64_t *words, uint64_t nwords),
                                  void *user, uint64_t *lists, uint64_t *consumed)
{
    return hec_seal_kswitch_keys_foreach_ex(bytes, nbytes, 0, visit, user, lists, consumed);
}

// KSwitchKeys::save of nlists key lists; list i has digits[i] PublicKeys of u64[2][K][N] (keys[i] = u64[L][2][K][N],
// NULL for an empty list).  parms_id = the key level's (all K moduli).
int hec_seal_kswitch_keys_save(uint64_t N, const uint64_t *coeff_modulus, uint64_t K, const uint64_t *const *keys,
                               const uint64_t *digits, uint64_t nlists, int compr_mode, void *out, uint64_t cap,
                               uint64_t *written)
{
    return io_guard([&] {
        if (!coeff_modulus || !K || (!keys && nlists) || (!digits && nlists)) throw std::invalid_argument("invalid argument");
        Writer m;
        u64 pid[4];
        parms_id_of(N, coeff_modulus, K, pid);
        m.bytes(pid, 32);
        m.put(nlists);
        for (u64 i = 0; i < nlists; ++i) {
            const u64 L = keys[i] ? digits[i] : 0;
            m.put(L);
            for (u64 j = 0; j < L; ++j) {
                CtData c;
                std::memcpy(c.parms_id, pid, 32);
                c.size = 2;
                c.level = K;
                c.N = N;
                c.scale = 1.0;
                c.data.assign(keys[i] + j * 2 * K * N, keys[i] + (j + 1) * 2 * K * N);
                Writer pk;
                emit_ciphertext(pk, c, 0);
                close_object(m, pk.b, 0);  // PublicKey wrapper
            }
        }
        Writer w;
        close_object(w, m.b, compr_mode);
        copy_out(w.b, out, cap, written);
    });
}

}  // extern "C"
