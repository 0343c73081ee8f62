// Internal host-side structures of the CKKS engine and the kernel launcher interface.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "hec_device.h"

namespace hec {

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
#define HEC_HIP(call)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess)                                                                  \
            throw ::hec::HipError(std::string(#call) + ": " + hipGetErrorString(e_));          \
    } while (0)

// Batched polynomial array: address(b, k, i) = p + b*sb + k*sk + i*N
struct PolyArr {
    u64 *p = nullptr;
    u64 sb = 0, sk = 0;
};

struct Ctx;

// Grow-only device scratch with named carving (no allocation inside steady-state launches).
struct Workspace {
    u64 *base = nullptr;
    std::size_t words = 0;
    // An outgrown base is retired, not freed: carved pointers of an enclosing Scratch and kernels already enqueued
    // may still use it.  It is reclaimed (stream drained, then hipFree) when the outermost Scratch of the context
    // ends; for batch lanes (defer_free) only by matvec_lanes after the lanes have joined, because a lane grows its
    // workspace from its own host thread while the other lanes are launching, and hipFree there (it synchronises
    // the device) coincided with rare wrong lanes at full size.  So a long-lived context does not accumulate them.
    bool defer_free = false;
    int depth = 0;  // live Scratch scopes on this workspace
    std::vector<u64 *> retired;
    void reserve(std::size_t w, hipStream_t stream);
    void reclaim(hipStream_t stream);
    void release();
};

struct Ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::size_t N = 0;
    int logN = 0;
    std::size_t K = 0, L = 0;
    std::vector<u64> q;             // host copy of the key moduli
    std::vector<DevPrime> hprimes;  // host copy
    std::vector<int> bits;
    DevPrime *primes = nullptr;     // device [K]
    ulonglong2 *tw = nullptr;       // device [K][N] {w, w_shoup}, w = psi^bitrev(idx)
    ulonglong2 *itw = nullptr;      // device [K][N] inverse twiddles psi^-bitrev(idx)
    ulonglong2 *twb = nullptr;      // device [K][N] pass-B layout of tw: [s][i][chunk] (see hec_kernels.hip)
    ulonglong2 *itwb = nullptr;     // same for itw
    double *twf = nullptr, *itwf = nullptr, *twbf = nullptr, *itwbf = nullptr;  // FP64 twins (q < 2^42)
    // device [K][N] w 2^31 mod q for the SEAL-ordered tw / itw (integer primes; the split-input Shoup butterflies of
    // the fan-out kernels, hec_device.h shoup_split_lazy), 0 at FP64 primes
    u64 *tws = nullptr, *itws = nullptr;
    u64 *twbs = nullptr;           // the same words for twb (pass-B layout; k_bmac's integer targets)
    bool bmac_split = true;        // HEC_BMAC_SPLIT=0: k_bmac's integer-target pass B on plain Shoup butterflies
    int nttb_shfl = 0;             // HEC_NTTB_SHFL=1: the forward NTT's pass B at N = 2^15 as k_nttb_shfl (exchanges
                                   // between lanes of a wavefront, no LDS tile), round 6
    int nt_e = 1;                  // the hoisted digits E stored non-temporally (round 6, +0.7 %; HEC_NT_E=0: cached)
    int moddown1 = 0;              // HEC_MODDOWN1=1: the single-pass mod-down (hec_moddown1.hip, N = 2^15)
    int hmac_int = 1;              // HEC_HMAC_INT=0: k_hmacm's 60-bit targets on the round-5 loop (gathered keys)
    int nttb_shfl_dr = 0;          // HEC_NTTB_SHFL_DR=1: the same for the divide-and-round pass B (A/B only)
    int split_bfly = 4;            // HEC_SPLIT_BFLY: 0 plain Shoup in the fan-out kernels, 1 split-input Shoup in
                                   // k_fan2, 2 also k_fan2j's per-thread-twiddle rounds, 3 all of k_fan2j, 4 k_fan2 and
                                   // k_fan2j's scalar-twiddle round (hec_kernels.hip run_fan; profiles/r05s_*)
    // key-switch target primes I in [0, l] (I == l is P) per level l, integer-arithmetic primes first:
    // device table imap + l * (HEC_MAXL + 2), built once at context creation; imap_nint[l] of them integer
    int *imap = nullptr;
    std::vector<int> imap_nint;
    const int *imap_at(int l) const { return imap + (std::size_t)l * (HEC_MAXL + 2); }
    // hoisted mod-up (see hec_kernels.hip): psi_i^e for e in [0, 2N) per key prime, c[J][I] = q_J mod q_I,
    // and a device flag raised when a digit limb holds more zero coefficients than the kernels correct
    u64 *psipow = nullptr;
    u64 *cji = nullptr;
    int *zflag = nullptr;           // [0] zero-list overflow, [1] debug count (HEC_DEBUG_LANES)
    int logR = 0;                   // pass split N = R x C, R = 2^ceil(logN/2)
    // CKKS encoder tables (hec_encode.hip), built on first encode: SEAL's matrix_reps_index_map_ (u32[N]) and
    // inv_root_powers_ (complex[N], entry 0 unused)
    u32 *enc_map = nullptr;
    double *enc_tw = nullptr;
    Workspace ws;
    // host-side constants
    std::vector<u64> p_inv, p_inv_q, p_half_mod;            // key switch mod-down (per data prime)
    std::vector<std::vector<u64>> ql_inv, ql_inv_q, ql_half_mod;  // rescale at level l (drop prime l-1)
    int tensor_defer_max = 12;     // HEC_TENSOR_DEFER: terminals per deferred tensor batch (1 = immediate)
    int tensor_defer_bufs = 8;     // HEC_TENSOR_BUFS: rotation buffers per trie depth
    int tensor_xcd = 0;            // HEC_TENSOR_XCD: k_tensor_multi2 grid in XCD clusters of this many batch groups
    bool hoist = true;             // HEC_HOIST=0: no hoisted mod-up in the rotation trie walk
    int hoist_min_children = 2;    // HEC_HOIST_MIN: children a trie node needs to be hoisted
    int hmac_cfg = 2;              // HEC_HMAC: 2 a sibling group per k_hmacm launch (slots of 2 children), 1 one
                                   // launch per sibling pair (round 4), 0 one hoisted MAC per child
    int hoist_scan = 1;            // HEC_HOIST_SCAN=0: hoisted node as INTT pass B, pass A, k_zscan, direct fan-out
                                   // (1: INTT pass B, then the fan-out finishes the INTT and lists the zeros)
    int hmac_odd3 = 1;             // HEC_HMAC_ODD3=0: an odd sibling group ends in a pair and a single-child launch
    bool fan_out = true;           // HEC_FAN=0: separate INTT pass A (fan-out fuses it into the forward passes A)
    // HEC_LANES: concurrent batch lanes of a matvec (hec_engine.hip matvec_lanes).  Opt-in since round 5: one lane
    // (the whole batch on the context's stream) is the default; 3 lanes measured +1.3 % at the bench's B = 192
    // (profiles/r05b_lanes_ab.json) but share the only unexplained full-size bit mismatch of rounds 2 and 4
    int lanes = 1;
    int lane_min_batch = 16;       // input vectors per lane at least
    bool fuse_galois = true;       // HEC_FUSE_GALOIS=0: materialise apply_galois before the key switch
    bool fused_modup_mac = true;  // HEC_FUSED_MODUP_MAC=0: separate mod-up pass B and key MAC kernels
    // HEC_POISON=1 (debug): every workspace carve (Scratch::take) and every freshly allocated output buffer is
    // filled with 0xFF bytes before use, so a kernel that reads memory this call never wrote sees a value no
    // residue can have (2^64 - 1; a NaN as FP64 bits) and the parity tests fail deterministically
    bool poison = false;
    bool lane_serial = false;      // HEC_LANE_SERIAL=1 (debug): the lanes run one after another, each drained
    // stream-ordered workspace fills and device-to-device copies as the engine's own kernels (k_fill32 / k_copy64) in
    // place of hipMemsetAsync / hipMemcpyAsync D2D.  Default since round 5: with the runtime calls, concurrent batch
    // lanes read a zero list whose fill had not landed (the round-2/4 bit mismatch);
    // HEC_KERNEL_MEMOPS=0 restores the runtime calls (A/B only)
    bool kernel_memops = true;
    bool debug_lanes = false;      // HEC_DEBUG_LANES=1 (debug): per call, report nodes with zero lists, the overflow
                                   // flag and changes of the per-key tables (stderr)
    // profiling (ProfScope in hec_engine.hip)
    int prof_mode = 0;  // 0 off, 1 synchronous per scope, 2 asynchronous event pairs
    // a scope's algorithmic bytes (compulsory reads + writes of its kernels) and kernel launches, so
    // per-kernel scopes ("k:<kernel>/<role>") give each kernel's achieved GB/s (bench.py roofline)
    struct ProfRec { double ms = 0; uint64_t n = 0; double bytes = 0; uint64_t kl = 0; };
    std::map<std::string, ProfRec> prof_tab;
    struct ProfPend { const char *name; hipEvent_t e0, e1; double bytes; int kl; };
    std::vector<ProfPend> prof_pend;
    std::vector<hipEvent_t> ev_pool;
    std::size_t ev_used = 0;
    int total_bits(std::size_t level) const
    {
        int b = 0;
        for (std::size_t i = 0; i < level; ++i) b += bits[i];
        return b;
    }
};

// ---------------------------------------------------------------- launchers (hec_kernels.hip)
// Batched NTT: job -> poly = job / nl, limb = job % nl; reads src + poly*ps_src + limb*N, writes
// dst + poly*ps_dst + limb*N (src may equal dst), prime = pmap[limb].
// elt != 1: the first pass loads src through the Galois permutation of elt (apply_galois_ntt fused).
// stages: 1 first pass only, 2 second pass only, 3 both.
void ntt_strided(Ctx &c, bool inverse, const u64 *src, u64 ps_src, u64 *dst, u64 ps_dst, int nl, const int *pmap,
                 int njobs, u32 elt = 1, int stages = 3);
// Key-switch phases (B targets at level l; see hec_engine.hip for the dataflow)
void ks_modup(Ctx &c, const u64 *D, u64 *E, int B, int l, int stages = 3,
              bool mform = false);  // stages as ntt_strided; mform: E in the MAC form k_hmacm reads
void ks_mac(Ctx &c, PolyArr T, const u64 *E, const u64 *key, u64 *ACC, int B, int l, u32 elt);
// fused: pass A of the mod-up NTTs (part & 1), then (pass B + key MAC) per target prime -> ACC[b][k][I]
// (part & 2)
void ks_modup_mac(Ctx &c, const u64 *D, u64 *E, PolyArr T, const u64 *key, u64 *ACC, int B, int l, int part,
                  u32 elt);
// divide-and-round by `last_idx` prime: Y = coefficient-form last limb per (b,k) (address Y + b*ysb + k*ysk),
// X / IN / OUT addressed (b,k,i), nk polys per batch entry, nl output limbs.
//   OUT = IN + (X - NTT(corr)) * inv   (IN optional; inv = last^-1 mod q_i)
// in_elt != 1: IN is read through the Galois permutation of in_elt
void divide_round(Ctx &c, const u64 *Y, u64 ysb, u64 ysk, PolyArr X, PolyArr IN, int in_nk, PolyArr OUT, int B,
                  int nk, int nl, int last_idx, const u64 *inv, const u64 *inv_q, u64 *Z, u32 in_elt = 1,
                  int stages = 3);
// fan-out kernels (see hec_kernels.hip): finish an INTT whose first pass ran (inverse pass A) and run
// the forward pass A of every target prime from registers.
//   mod-up:  D[b][J] -> E[b][I][J] (I != J), the input of k_bmac / ks_modup's pass B
//   mod-down: last limb (b, k) at Y + b ysb + k ysk -> Z[b][k][i], the input of divide_round pass B
// zl (non-direct only): also list the zero coefficients of the INTT's canonical values (zero_scan's format)
void fan_modup(Ctx &c, const u64 *D, u64 *E, int B, int l, bool direct = false, int *zl = nullptr);
// hoisted mod-up (hec_kernels.hip): zero_scan lists the zero coefficients of nlimbs canonical limbs
// (zl: per limb count + HEC_ZCAP positions; more raises c.zflag); hoisted_mac is one child's key MAC
// from the node's NTT-form digits E, the child's sign-mask NTTs W (K limbs) and X1 = the node's c1.
#define HEC_ZCAP 8
void zero_scan(Ctx &c, const u64 *D, int nlimbs, int *zl);
void debug_count_zl(Ctx &c, const int *zl, int *cnt);  // HEC_DEBUG_LANES: ++*cnt when zl[0] != 0
// stream-ordered device fill / copy as engine kernels; dev_fill / dev_zero use them when c.kernel_memops, else the
// runtime's hipMemsetAsync
void dev_fill32(Ctx &c, void *p, u32 v, std::size_t bytes);
void dev_copy64(Ctx &c, u64 *dst, const u64 *src, std::size_t words);
void dev_fill(Ctx &c, void *p, u32 v, std::size_t bytes);
void dev_zero(Ctx &c, void *p, std::size_t bytes);
void hoisted_mac(Ctx &c, PolyArr X1, const u64 *E, const u64 *W, const int *zl, const u64 *key, u64 *ACC, int B,
                 int l, u32 elt);
// the same for up to 4 sibling rotations at once (the node's digits read once for all of them)
struct HChildSpec {
    u32 elt, einv;  // Galois element and its inverse mod 2N
    const u64 *key, *W;
    u64 *ACC;
    const u64 *KW;  // key_wsum of the child's key at this level
    const u64 *MK;  // the child's key in MAC form and source order (mac_key_table)
};
// MK[J][k][I][s] = the key word at the child's output position galois_src(s, einv), FP64-class limbs as double bits,
// 60-bit limbs as lo30 | hi30 << 32 (hec_kernels.hip, the MAC form of k_hmacm)
void mac_key_table(Ctx &c, const u64 *key, u64 *MK, u32 einv);
constexpr int HMAC_MAX_CHILDREN = 6;  // largest hoisted_group()
// KW[k][I] = sum_{J<l, J!=I} (q_J mod q_I) key[J][k][I] mod q_I, I in [0, l] (I == l: P), k in {0, 1}
void key_wsum(Ctx &c, const u64 *key, u64 *KW, int l);
void hoisted_mac_multi(Ctx &c, PolyArr X1, PolyArr X0, const u64 *E, const int *zl, const HChildSpec *kids, int nkids,
                       int B, int l);
// three children in one sibling-fused launch (3 x 4 FP64 / 3 x 2 integer batch entries per thread)
void hoisted_mac_3(Ctx &c, PolyArr X1, PolyArr X0, const u64 *E, const int *zl, const HChildSpec *kids, int B, int l);
// a whole sibling group (up to HMAC_MAX_CHILDREN) in one launch: slots of 2 children, the digit tile shared through L2
void hoisted_mac_group(Ctx &c, PolyArr X1, PolyArr X0, const u64 *E, const int *zl, const HChildSpec *kids, int nkids,
                       int B, int l);
int hoisted_group(const Ctx &c);  // children per hoisted_mac_multi call for c.hmac_cfg
void fan_divide_round(Ctx &c, const u64 *Y, u64 ysb, u64 ysk, u64 *Z, int B, int nk, int nl, int last_idx);
// the single-pass mod-down (hec_moddown1.hip): Y the coefficient-form special-prime limbs, X the ACC data limbs;
// false when it does not apply (N != 2^15)
bool moddown1(Ctx &c, const u64 *Y, u64 ysb, u64 ysk, PolyArr X, PolyArr IN, int in_nk, PolyArr OUT, int B, int nk,
              int nl, int last_idx, u32 elt);
void galois_permute(Ctx &c, PolyArr in, PolyArr out, int B, int nk, int nl, u32 elt);
void tensor_acc(Ctx &c, PolyArr R, const u64 *A, u64 a_sk, PolyArr ACC, int B, int l, bool assign);
// deferred tensor products: ACC[b] (=|+=) sum_t R_t[b] (x) A_t, T <= TB_MAX rotated inputs
// (R_t[b] at r[t] + b r_sb, polys r_sk apart; A_t polys a_sk apart)
constexpr int TB_MAX = 12;
struct TensorBatch {
    const u64 *r[TB_MAX];
    const u64 *a[TB_MAX];
    int T;
};
void tensor_multi(Ctx &c, const TensorBatch &tb, u64 r_sb, u64 r_sk, u64 a_sk, PolyArr ACC, int B, int l,
                  bool assign, bool plain = false);  // plain: the A_t are plaintexts (ct x pt, 2-poly ACC)
void tensor_sum(Ctx &c, PolyArr R, PolyArr A, u64 *ACC, u64 acc_sk, int B, int l);
void ew_add(Ctx &c, PolyArr a, PolyArr b, PolyArr out, int B, int nk, int nl, int mode);  // 0 add, 1 sub
void ew_negate(Ctx &c, PolyArr a, int B, int nk, int nl);
void ew_mul_plain(Ctx &c, PolyArr a, const u64 *pt, int nk, int nl);
void ew_dyadic(Ctx &c, const u64 *a, const u64 *b, u64 *out, int limb0, int nl, int npolys);
void ct_multiply(Ctx &c, const u64 *a, int sa, const u64 *b, int sb, u64 *out, int nl);
void ew_reduce(Ctx &c, u64 *p, int npoly, int nl);
void fill_uniform(Ctx &c, u64 *p, int npoly, int nl, int limb_prime0, int special_last, u64 seed);
// p[i][*] = words[i] for the nl limbs (a scalar plaintext in NTT form)
void fill_limbs(Ctx &c, u64 *p, int nl, const u64 *words);
// CKKS encode of `count` slot vectors (hec_encode.hip): re/im device [count][nv] (im may be null), work
// device doubles [count][2N], out [count][level][N] NTT form, maxabs[count] = max |coefficient| (bits
// of a double)
void encode_batch(Ctx &c, const double *re, const double *im, u64 nv, int count, double scale, int level, double *work,
                  u64 *out, u64 *maxabs);

}  // namespace hec
