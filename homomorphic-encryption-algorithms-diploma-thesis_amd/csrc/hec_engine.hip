// Host orchestration + C-ABI of the CKKS engine (include/hecdna.h).
//
// Every public entry point restates one seal::Evaluator call that the reference's he_operators /
// he_linalg layer makes (file:line cited per function in hecdna.h), on device-resident SEAL-layout
// objects.  Internally all ciphertext work is BATCHED: the key switch, rotation and rescale
// routines take B ciphertexts in one strided array so that one launch sequence (and one read of
// the key) serves the whole batch; the single-object C-ABI calls are the B = 1 case.
//
// Key switch dataflow (SEAL 4.1 Evaluator::switch_key_inplace, per-prime digits + special prime P,
// SURVEY §8(a) a5), B targets T[b] (NTT form, l limbs):
//   (1) D[b][J]    = INTT_J(T[b][J])                                    ntt_strided (inverse)
//   (2) E[b][I][J] = NTT_I(D[b][J] mod q_I),  I in {0..l-1, P}, I != J   ks_modup (reduction fused)
//   (3) ACC[b][k][I] = sum_J E[b][I][J] * key[J][k][I]   (E[b][I][I] = T[b][I])   ks_mac
//   (4) y = INTT_P(ACC[b][k][P])                                        ntt_strided (inverse)
//   (5) OUT[b][k][i] = IN[b][k][i] + (ACC[b][k][i] - NTT_i(round(y))) * P^-1     divide_round
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <limits>
#include <mutex>
#include <set>
#include <thread>
#include <tuple>

#include "hec_internal.h"

#include <dlfcn.h>
#include <unistd.h>
#include <rccl/rccl.h>
#include "hecdna.h"

using namespace hec;
using u128 = unsigned __int128;

// =============================================================================== objects ===
// The communicator of the sharded matvec (one process per GPU): RCCL over xGMI (hec_comm_init) or a caller's host
// collectives (hec_comm_init_ops).  shard_agree needs only allreduce_f64; the data exchange sums the ranks' partial
// accumulators in u64.
struct HecComm {
    virtual ~HecComm() = default;
    // in place over the world, host memory: op HEC_REDUCE_MIN / HEC_REDUCE_MAX
    virtual void allreduce_f64(double *host, std::size_t n, int op, hipStream_t s) = 0;
    // in place over the world, a device buffer ordered on stream s: the sum (exact: world <= 8, residues < 2^60)
    virtual void allreduce_u64_sum(u64 *dev, std::size_t n, hipStream_t s) = 0;
};
struct hec_context {
    Ctx c;
    // batch lanes (matvec_lanes): contexts sharing this one's device tables, each with its own HIP
    // stream, workspace and zero flag, built on first use
    std::vector<hec_context *> lanes;
    // persistent events of matvec_lanes (created with the first lane, destroyed with the context): the lanes
    // wait on lanes_start, the context stream waits on each lane's lane_done.  An event destroyed right after
    // a hipStreamWaitEvent on it could let that wait pass early (a rare whole-lane race seen at full size).
    hipEvent_t lanes_start = nullptr, lane_done = nullptr;
    // multi-GPU (hec_comm_init): this process's rank in a world of one process per GPU, RCCL communicator
    int rank = 0, world = 1;
    HecComm *comm = nullptr;
    u64 gen = 0;  // this context's entry in the live-context registry (ctx_alive)
};
// Objects may outlive their context (SEAL's objects hold their context by shared_ptr, so a caller may free them in
// any order, and a garbage collector finalising a reference cycle picks its own order): every object records its
// context's generation, and its destroy touches the context (device, stream) only while that context is alive.
// An address reused by a later context carries a new generation, so it is never mistaken for the old one.
static std::mutex g_live_mu;
static std::map<const hec_context *, u64> g_live;
static u64 g_live_gen = 0;
static u64 ctx_register(const hec_context *c)
{
    std::lock_guard<std::mutex> lock(g_live_mu);
    return g_live[c] = ++g_live_gen;
}
static void ctx_unregister(const hec_context *c)
{
    std::lock_guard<std::mutex> lock(g_live_mu);
    g_live.erase(c);
}
static bool ctx_alive(const hec_context *c, u64 gen)
{
    std::lock_guard<std::mutex> lock(g_live_mu);
    const auto it = g_live.find(c);
    return c && it != g_live.end() && it->second == gen;
}
struct hec_ciphertext {
    hec_context *ctx = nullptr;
    u64 ctx_gen = 0;
    u64 *d = nullptr;
    std::size_t cap = 0;  // words
    std::size_t size = 0, level = 0;
    double scale = 1.0;
};
struct hec_plaintext {
    hec_context *ctx = nullptr;
    u64 ctx_gen = 0;
    u64 *d = nullptr;
    std::size_t cap = 0;
    std::size_t level = 0;
    double scale = 1.0;
};
struct hec_kswitch_key {
    hec_context *ctx = nullptr;
    u64 ctx_gen = 0;
    u64 *d = nullptr;
};
struct hec_galois_keys {
    hec_context *ctx = nullptr;
    u64 ctx_gen = 0;
    std::map<u32, u64 *> keys;
    std::map<u32, u64 *> negw;  // hoisted mod-up: W_elt[I] = NTT_I(sign mask of elt), built on first use
    // hoisted MAC: KW[elt, l][k][I] = sum_{J<l, J!=I} (q_J mod q_I) key_elt[J][k][I] mod q_I, built on first
    // use per level, dropped when the key is replaced
    std::map<std::pair<u32, int>, u64 *> kw;
    std::map<u32, u64 *> mkey;  // hoisted MAC: the key in MAC form and source order (mac_key_table), first use
    void drop_kw(u32 elt)  // the tables derived from the key's words (KW at every level, MK)
    {
        if (auto m = mkey.find(elt); m != mkey.end()) {
            (void)hipFree(m->second);
            mkey.erase(m);
        }
        for (auto it = kw.begin(); it != kw.end();) {
            if (it->first.first == elt) {
                (void)hipFree(it->second);
                it = kw.erase(it);
            } else {
                ++it;
            }
        }
    }
};

namespace {

thread_local std::string g_err;

template <class F>
int guard(F &&f)
{
    try {
        f();
        return HEC_OK;
    } catch (const HipError &e) {
        g_err = e.what();
        return HEC_EDEVICE;
    } catch (const std::invalid_argument &e) {
        g_err = e.what();
        return HEC_EINVAL;
    } catch (const std::logic_error &e) {
        g_err = e.what();
        return HEC_ELOGIC;
    } catch (const std::exception &e) {
        g_err = e.what();
        return HEC_EDEVICE;
    }
}

void need(bool cond, const char *msg)
{
    if (!cond) throw std::invalid_argument(msg);
}

// ------------------------------------------------------------------ host number theory -----
u64 powm(u64 b, u64 e, u64 q)
{
    u64 r = 1 % q;
    b %= q;
    for (; e; e >>= 1) {
        if (e & 1) r = (u64)((u128)r * b % q);
        b = (u64)((u128)b * b % q);
    }
    return r;
}
u64 invm(u64 a, u64 q)
{
    __int128 t = 0, nt = 1, r = q, nr = a % q;
    while (nr) {
        const __int128 k = r / nr;
        __int128 x = t - k * nt; t = nt; nt = x;
        x = r - k * nr; r = nr; nr = x;
    }
    if (r != 1) throw std::invalid_argument("value is not invertible");
    return (u64)(t < 0 ? t + q : t);
}
bool isprime(u64 n)
{
    if (n < 2) return false;
    static const u64 sp[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (u64 p : sp) {
        if (n % p == 0) return n == p;
    }
    u64 d = n - 1;
    int s = 0;
    while (!(d & 1)) { d >>= 1; ++s; }
    for (u64 a : sp) {
        u64 x = powm(a, d, n);
        if (x == 1 || x == n - 1) continue;
        bool composite = true;
        for (int i = 1; i < s && composite; ++i) {
            x = (u64)((u128)x * x % n);
            if (x == n - 1) composite = false;
        }
        if (composite) return false;
    }
    return true;
}
u64 shoupq(u64 w, u64 q) { return (u64)(((u128)w << 64) / q); }
u32 brev(u32 x, int bits)
{
    u32 r = 0;
    for (int i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
    return r;
}
// SEAL util::try_minimal_primitive_root: the smallest primitive 2N-th root of unity mod q
u64 minimal_root(u64 two_n, u64 q)
{
    u64 g = 0;
    for (u64 x = 2; x < q && !g; ++x) {
        const u64 c = powm(x, (q - 1) / two_n, q);
        if (powm(c, two_n / 2, q) == q - 1) g = c;
    }
    if (!g) throw std::logic_error("no primitive root found");
    const u64 g2 = (u64)((u128)g * g % q);
    u64 cur = g, best = g;
    for (u64 k = 0; k < two_n / 2; ++k) {
        best = std::min(best, cur);
        cur = (u64)((u128)cur * g2 % q);
    }
    return best;
}
bool are_close(double a, double b)  // SEAL util::are_close
{
    const double sf = std::max({std::fabs(a), std::fabs(b), 1.0});
    return std::fabs(a - b) < std::numeric_limits<double>::epsilon() * sf;
}
bool scale_ok(const Ctx &c, double scale, std::size_t level)  // SEAL is_scale_within_bounds
{
    return !(scale <= 0 || (int)std::log2(scale) >= c.total_bits(level));
}
std::vector<int> naf(int value)  // SEAL util::naf: least-significant term first
{
    std::vector<int> res;
    const bool sign = value < 0;
    value = std::abs(value);
    for (int i = 0; value; ++i) {
        const int zi = (value & 1) ? 2 - (value & 3) : 0;
        value = (value - zi) >> 1;
        if (zi) res.push_back((sign ? -zi : zi) * (1 << i));
    }
    return res;
}
u32 elt_from_step(const Ctx &c, int step)  // SEAL GaloisTool::get_elt_from_step
{
    const u32 n = (u32)c.N, m = 2 * n;
    if (step == 0) return m - 1;
    const bool sign = step < 0;
    u32 pos = (u32)std::abs(step);
    if (pos >= (n >> 1)) throw std::invalid_argument("step count too large");
    pos &= m - 1;
    int s = sign ? (int)(n >> 1) - (int)pos : (int)pos;
    u64 elt = 1;
    while (s--) { elt *= 3; elt &= m - 1; }
    return (u32)elt;
}
// SEAL Evaluator::rotate_internal flattened into the sequence of Galois elements it applies
void rotation_elts(const Ctx &c, int steps, const hec_galois_keys &gk, std::vector<u32> &out)
{
    if (steps == 0) return;
    const u32 elt = elt_from_step(c, steps);
    if (gk.keys.count(elt)) { out.push_back(elt); return; }
    const std::vector<int> terms = naf(steps);
    if (terms.size() == 1) throw std::invalid_argument("Galois key not present");
    for (int s : terms)
        if ((std::size_t)std::abs(s) != (c.N >> 1)) rotation_elts(c, s, gk, out);
}

// ------------------------------------------------------------------ device memory ----------
u64 *dalloc(std::size_t words)
{
    void *p = nullptr;
    if (words == 0) words = 1;
    HEC_HIP(hipMalloc(&p, words * sizeof(u64)));
    return (u64 *)p;
}
void ensure(hec_ciphertext *ct, std::size_t words)
{
    if (ct->cap >= words) return;
    if (ct->d) HEC_HIP(hipFree(ct->d));
    ct->d = dalloc(words);
    ct->cap = words;
    if (ct->ctx && ct->ctx->c.poison) dev_fill(ct->ctx->c, ct->d, 0xFFFFFFFFu, words * sizeof(u64));
}

// stack-style carving of the context workspace; kernels are stream ordered, so a region released
// here may be reused by the next enqueued operation.
struct Scratch {
    Ctx &c;
    std::size_t top = 0;
    explicit Scratch(Ctx &cc, std::size_t words) : c(cc)
    {
        c.ws.reserve(words, c.stream);
        ++c.ws.depth;
    }
    ~Scratch()
    {
        if (--c.ws.depth == 0 && !c.ws.defer_free && !c.ws.retired.empty()) {
            try {
                c.ws.reclaim(c.stream);
            } catch (...) {  // keep them for release(); a destructor must not throw
            }
        }
    }
    Scratch(const Scratch &) = delete;
    Scratch &operator=(const Scratch &) = delete;
    u64 *take(std::size_t w)
    {
        w = (w + 63) & ~(std::size_t)63;
        if (top + w > c.ws.words) throw std::logic_error("workspace overflow");
        u64 *p = c.ws.base + top;
        top += w;
        if (c.poison) dev_fill(c, p, 0xFFFFFFFFu, w * sizeof(u64));
        return p;
    }
};

// ------------------------------------------------------------------ profiling -------------
// Per-class GPU time of the engine's phases.  prof_mode 1: event pair + synchronize per scope;
// prof_mode 2: event pairs from a reusable pool recorded asynchronously (no host sync inside the
// call), resolved when the profile is read.
struct ProfScope {
    Ctx &c;
    const char *name;
    double bytes = 0;
    int kl = 1;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    hipEvent_t pool_event()
    {
        if (c.ev_used == c.ev_pool.size()) {
            hipEvent_t e;
            HEC_HIP(hipEventCreate(&e));
            c.ev_pool.push_back(e);
        }
        return c.ev_pool[c.ev_used++];
    }
    ProfScope(Ctx &cc, const char *n, double limbs = 0, int launches = 1)
        : c(cc), name(n), bytes(limbs * 8.0 * (double)cc.N), kl(launches)
    {
        if (!c.prof_mode) return;
        if (c.prof_mode == 2) {
            e0 = pool_event();
            e1 = pool_event();
        } else {
            HEC_HIP(hipEventCreate(&e0));
            HEC_HIP(hipEventCreate(&e1));
        }
        HEC_HIP(hipEventRecord(e0, c.stream));
    }
    ~ProfScope()
    {
        if (!c.prof_mode || !e0) return;
        (void)hipEventRecord(e1, c.stream);
        if (c.prof_mode == 2) {
            c.prof_pend.push_back({name, e0, e1, bytes, kl});
            return;
        }
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        auto &r = c.prof_tab[name];
        r.ms += ms;
        r.n += 1;
        r.bytes += bytes;
        r.kl += kl;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
};
void prof_resolve(Ctx &c)
{
    if (c.prof_pend.empty()) return;
    HEC_HIP(hipStreamSynchronize(c.stream));
    for (const auto &p : c.prof_pend) {
        float ms = 0;
        HEC_HIP(hipEventElapsedTime(&ms, p.e0, p.e1));
        auto &r = c.prof_tab[p.name];
        r.ms += ms;
        r.n += 1;
        r.bytes += p.bytes;
        r.kl += p.kl;
    }
    c.prof_pend.clear();
    c.ev_used = 0;
}

// ------------------------------------------------------------------ batched building blocks
std::size_t ks_words(const Ctx &c, std::size_t B, std::size_t l)
{
    return c.N * B * (l + (l + 1) * l + 2 * (l + 1) + 2 * l) + 4 * 64;
}

// key-switch mod-down (SEAL switch_key_inplace step 4): the P-limb INTT's first pass, the fan-out that
// finishes it and forms the rounding limbs, and divide_round's pass B (OUT = IN + (ACC_i - r) P^-1)
// single-pass form (c.moddown1, N = 2^15): the P limbs' whole INTT in place, then k_moddown1 forms each data limb's
// rounding limb, transforms it and divides-and-rounds in one kernel (no Z round trip, no fan-out, no pass B)
static bool moddown_single(Ctx &c, u64 *ACC, PolyArr IN, int in_nk, const PolyArr *OUT, const u32 *elts, int ng, int B,
                           int l)
{
    if (!c.moddown1 || c.logN != 15) return false;
    const u64 N = c.N, sacc = (u64)B * 2 * (l + 1) * N;
    ProfScope ps(c, "ks_moddown");
    const int pP[1] = {(int)c.K - 1};
    {  // both passes of the P limbs' INTT: read + write 2 B ng limbs per pass
        ProfScope k(c, "k:k_ntt/moddown_intt", 8.0 * B * ng, 2);
        ntt_strided(c, true, ACC + l * N, (l + 1) * N, ACC + l * N, (l + 1) * N, 1, pP, 2 * B * ng, 1, 3);
    }
    for (int q = 0; q < ng; ++q) {  // P limb (2B, once per (b, k)), ACC (2Bl), IN (in_nk B l), OUT (2Bl)
        ProfScope k(c, "k:k_moddown1/moddown", (2.0 + (4.0 + in_nk) * l) * B, 2);  // one launch per class
        moddown1(c, ACC + q * sacc + l * N, 2 * (l + 1) * N, (l + 1) * N, PolyArr{ACC + q * sacc, 2 * (l + 1) * N, (l + 1) * N},
                 IN, in_nk, OUT[q], B, 2, l, (int)c.K - 1, elts[q]);
    }
    return true;
}

void moddown(Ctx &c, u64 *ACC, u64 *Z, PolyArr IN, int in_nk, PolyArr OUT, int B, int l, u32 elt)
{
    if (moddown_single(c, ACC, IN, in_nk, &OUT, &elt, 1, B, l)) return;
    const u64 N = c.N;
    const bool fan = c.fan_out;
    ProfScope ps(c, "ks_moddown");
    const int pP[1] = {(int)c.K - 1};
    {  // P limbs of both key polys: read + write 2B limbs per pass
        ProfScope k(c, fan ? "k:k_ntt/moddown_intt" : "k:k_ntt/moddown_intt2", 4.0 * B, fan ? 1 : 2);
        ntt_strided(c, true, ACC + l * N, (l + 1) * N, ACC + l * N, (l + 1) * N, 1, pP, 2 * B, 1, fan ? 1 : 3);
    }
    if (fan) {  // 2B P limbs -> 2B l rounding limbs (pass-A domain)
        ProfScope k(c, "k:k_fan2/moddown", 2.0 * B * (l + 1));
        fan_divide_round(c, ACC + l * N, 2 * (l + 1) * N, (l + 1) * N, Z, B, 2, l, (int)c.K - 1);
    }
    {  // Z (2Bl), ACC data limbs (2Bl), IN (in_nk B l), OUT (2Bl)
        ProfScope k(c, fan ? "k:k_ntt/divround_b" : "k:k_ntt/divround2", (6.0 + in_nk) * B * l, fan ? 1 : 2);
        divide_round(c, ACC + l * N, 2 * (l + 1) * N, (l + 1) * N, PolyArr{ACC, 2 * (l + 1) * N, (l + 1) * N}, IN,
                     in_nk, OUT, B, 2, l, (int)c.K - 1, c.p_inv.data(), c.p_inv_q.data(), Z, elt, fan ? 2 : 3);
    }
}

// The mod-downs of ng sibling rotations of one node at once: ACC[q] = ACC + q B 2 (l+1) N (contiguous), IN the
// node's ciphertexts read through each child's permutation.  The P-limb INTT pass and the fan-out (small,
// latency-bound launches) run over all ng B entries in one launch each; divide_round's pass B per child.
void moddown_group(Ctx &c, u64 *ACC, u64 *Z, PolyArr IN, int in_nk, const PolyArr *OUT, const u32 *elts, int ng,
                   int B, int l)
{
    const u64 N = c.N, sacc = (u64)B * 2 * (l + 1) * N, sz = (u64)B * 2 * l * N;
    if (moddown_single(c, ACC, IN, in_nk, OUT, elts, ng, B, l)) return;
    if (!c.fan_out || ng == 1) {
        for (int q = 0; q < ng; ++q) moddown(c, ACC + q * sacc, Z, IN, in_nk, OUT[q], B, l, elts[q]);
        return;
    }
    ProfScope ps(c, "ks_moddown");
    const int pP[1] = {(int)c.K - 1};
    {
        ProfScope k(c, "k:k_ntt/moddown_intt", 4.0 * B * ng);
        ntt_strided(c, true, ACC + l * N, (l + 1) * N, ACC + l * N, (l + 1) * N, 1, pP, 2 * B * ng, 1, 1);
    }
    {
        ProfScope k(c, "k:k_fan2/moddown", 2.0 * B * ng * (l + 1));
        fan_divide_round(c, ACC + l * N, 2 * (l + 1) * N, (l + 1) * N, Z, B * ng, 2, l, (int)c.K - 1);
    }
    for (int q = 0; q < ng; ++q) {
        ProfScope k(c, "k:k_ntt/divround_b", (6.0 + in_nk) * B * l);
        divide_round(c, ACC + q * sacc + l * N, 2 * (l + 1) * N, (l + 1) * N,
                     PolyArr{ACC + q * sacc, 2 * (l + 1) * N, (l + 1) * N}, IN, in_nk, OUT[q], B, 2, l, (int)c.K - 1,
                     c.p_inv.data(), c.p_inv_q.data(), Z + q * sz, elts[q], 2);
    }
}

// T (the target polys) and IN (added to the output) are read through the Galois permutation of elt
// (elt = 1: as they are).  OUT must not overlap T or IN when elt != 1 (the reads gather).
void keyswitch(Ctx &c, Scratch &s, PolyArr T, const u64 *key, PolyArr IN, int in_nk, PolyArr OUT, int B, int l,
               u32 elt = 1)
{
    const u64 N = c.N;
    const std::size_t top = s.top;
    u64 *D = s.take(B * l * N), *E = s.take((u64)B * (l + 1) * l * N), *ACC = s.take((u64)B * 2 * (l + 1) * N),
        *Z = s.take((u64)B * 2 * l * N);
    int pmap[HEC_MAXL + 1];
    for (int i = 0; i <= HEC_MAXL; ++i) pmap[i] = i;
    const bool fan = c.fan_out && c.fused_modup_mac;
    const double K = l + 1;
    {
        ProfScope ps(c, "ks_intt");  // with fan-out only its first pass; the fan kernel finishes it
        ProfScope k(c, fan ? "k:k_ntt/intt_b" : "k:k_ntt/intt2", 2.0 * B * l, fan ? 1 : 2);
        ntt_strided(c, true, T.p, T.sb, D, l * N, l, pmap, B * l, elt, fan ? 1 : 3);
    }
    if (c.fused_modup_mac) {  // mod-up pass A, then pass B fused with the key MAC (no E round trip)
        {
            ProfScope ps(c, "ks_modup_a");
            ProfScope k(c, fan ? "k:k_fan2j/modup" : "k:k_ntt/modup_a", (double)B * l * (l + 1), 1);
            if (fan) fan_modup(c, D, E, B, l);
            else ks_modup_mac(c, D, E, T, key, ACC, B, l, 1, elt);
        }
        {  // digits E (B l^2) + the I == J targets (B l) + key (2 l K) -> ACC (2 B K)
            ProfScope ps(c, "ks_bmac");
            ProfScope k(c, "k:k_bmac", (double)B * l * l + (double)B * l + 2.0 * l * K + 2.0 * B * K,
                        1);
            ks_modup_mac(c, D, E, T, key, ACC, B, l, 2, elt);
        }
    } else {
        {
            ProfScope ps(c, "ks_modup");
            ks_modup(c, D, E, B, l);
        }
        {
            ProfScope ps(c, "ks_mac");
            ks_mac(c, T, E, key, ACC, B, l, elt);
        }
    }
    moddown(c, ACC, Z, IN, in_nk, OUT, B, l, elt);
    s.top = top;
}

// hoisted mod-up data of one trie node (B targets at level l): D = INTT(c1) (canonical coefficient form),
// E[b][I][J] = NTT_I(D_J mod q_I) (canonical NTT form, J != I), zero lists of D (see hec_kernels.hip)
constexpr int HOIST_GROUP = 6;  // sibling rotations per grouped mod-down (and per k_hmacm accumulator set)
struct Hoist {
    u64 *D = nullptr, *E = nullptr;
    int *zl = nullptr;
    // key-switch accumulators of up to HOIST_GROUP siblings, contiguous (moddown_group), live across the recursion
    // into their subtrees
    u64 *acc0 = nullptr;
    u64 sacc = 0;
    u64 *acc(int q) const { return acc0 + (u64)q * sacc; }
};
std::size_t hoist_words(const Ctx &c, std::size_t B, std::size_t l)
{
    return c.N * B * (l + (l + 1) * l + (std::size_t)HOIST_GROUP * 2 * (l + 1)) +
           ((1 + B * l * (HEC_ZCAP + 1)) * sizeof(int) + 7) / 8 + 4 * 64;
}
Hoist hoist_alloc(const Ctx &c, Scratch &s, int B, int l)
{
    Hoist h;
    h.D = s.take((u64)B * l * c.N);
    h.E = s.take((u64)B * (l + 1) * l * c.N);
    h.zl = reinterpret_cast<int *>(s.take(((1 + (u64)B * l * (HEC_ZCAP + 1)) * sizeof(int) + 7) / 8));
    h.sacc = (u64)B * 2 * (l + 1) * c.N;
    h.acc0 = s.take((u64)HOIST_GROUP * h.sacc);
    return h;
}
void hoist_node(Ctx &c, PolyArr X, int B, int l, const Hoist &h)
{
    const u64 N = c.N;
    int pmap[HEC_MAXL + 1];
    for (int i = 0; i <= HEC_MAXL; ++i) pmap[i] = i;
    if (c.hoist_scan) {  // the fan-out finishes the INTT and lists the zeros: no D round trip
        {
            ProfScope ps(c, "ks_intt");
            ProfScope k(c, "k:k_ntt/intt_b", 2.0 * B * l);
            ntt_strided(c, true, X.p + X.sk, X.sb, h.D, l * N, l, pmap, B * l, 1, 1);
        }
        ProfScope ps(c, "ks_modup_h");
        {
            ProfScope k(c, "k:k_fan2j/hoist", (double)B * l * (l + 1));
            fan_modup(c, h.D, h.E, B, l, false, h.zl);
        }
        ProfScope k(c, "k:k_ntt/modup_h_b", 2.0 * B * l * l);
        ks_modup(c, h.D, h.E, B, l, 2, c.hmac_cfg != 0);  // pass B: NTT-form digits (k_hmacm: MAC form)
        return;
    }
    {
        ProfScope ps(c, "ks_intt");
        {
            ProfScope k(c, "k:k_ntt/intt_b", 2.0 * B * l);
            ntt_strided(c, true, X.p + X.sk, X.sb, h.D, l * N, l, pmap, B * l, 1, 1);
        }
        {
            ProfScope k(c, "k:k_ntt/intt_a", 2.0 * B * l);
            ntt_strided(c, true, h.D, l * N, h.D, l * N, l, pmap, B * l, 1, 2);
        }
        ProfScope k(c, "k:k_zscan", (double)B * l);
        zero_scan(c, h.D, B * l, h.zl);
    }
    ProfScope ps(c, "ks_modup_h");
    {
        ProfScope k(c, "k:k_fan2j/hoist", (double)B * l * (l + 1));
        fan_modup(c, h.D, h.E, B, l, true);  // pass A of every NTT_I(D_J mod q_I), from the canonical D
    }
    ProfScope k(c, "k:k_ntt/modup_h_b", 2.0 * B * l * l);
    ks_modup(c, h.D, h.E, B, l, 2, c.hmac_cfg != 0);  // pass B: NTT-form digits (k_hmacm: MAC form)
}
// one child of a hoisted node: OUT = key switch of apply_galois(X, elt) (X: the node's ciphertexts)
void hoisted_child(Ctx &c, Scratch &s, PolyArr X, const Hoist &h, const u64 *W, const u64 *key, PolyArr OUT, int B,
                   int l, u32 elt)
{
    const u64 N = c.N;
    const std::size_t top = s.top;
    u64 *ACC = s.take((u64)B * 2 * (l + 1) * N), *Z = s.take((u64)B * 2 * l * N);
    {
        ProfScope ps(c, "ks_hmac");
        hoisted_mac(c, PolyArr{X.p + X.sk, X.sb, 0}, h.E, W, h.zl, key, ACC, B, l, elt);
    }
    moddown(c, ACC, Z, PolyArr{X.p, X.sb, X.sk}, 1, OUT, B, l, elt);
    s.top = top;
}
std::size_t hoisted_child_words(const Ctx &c, std::size_t B, std::size_t l)
{
    return c.N * B * std::max(2 * (l + 1) + 2 * l, (std::size_t)HOIST_GROUP * 2 * l) + 2 * 64;
}

// the sign-mask NTTs of a Galois key (built on first use): W[I] = NTT_I(m), m[t] = 1 iff coefficient t of
// apply_galois(x, elt) is a negated coefficient of x, i.e. t elt^-1 mod 2N >= N
const u64 *galois_negw(hec_context *ctx, hec_galois_keys &gk, u32 elt)
{
    auto it = gk.negw.find(elt);
    if (it != gk.negw.end()) return it->second;
    Ctx &c = ctx->c;
    const u64 N = c.N, m2 = 2 * N;
    const u64 einv = invm(elt, m2);
    std::vector<u64> mask(c.K * N);
    for (u64 t = 0; t < N; ++t) mask[t] = ((t * einv) % m2) >= N ? 1 : 0;
    for (std::size_t i = 1; i < c.K; ++i) std::copy(mask.begin(), mask.begin() + N, mask.begin() + i * N);
    u64 *W = dalloc(c.K * N);
    HEC_HIP(hipMemcpyAsync(W, mask.data(), c.K * N * sizeof(u64), hipMemcpyHostToDevice, c.stream));
    int pmap[HEC_MAXL + 1];
    for (int i = 0; i <= HEC_MAXL; ++i) pmap[i] = i;
    ntt_strided(c, false, W, c.K * N, W, c.K * N, (int)c.K, pmap, (int)c.K);
    HEC_HIP(hipStreamSynchronize(c.stream));  // the host mask goes out of scope
    gk.negw[elt] = W;
    return W;
}

// the sign-mask key sums of a Galois key at level l (built on first use, see k_keyw)
const u64 *galois_kw(hec_context *ctx, hec_galois_keys &gk, u32 elt, int l)
{
    auto it = gk.kw.find({elt, l});
    if (it != gk.kw.end()) return it->second;
    Ctx &c = ctx->c;
    u64 *KW = dalloc((std::size_t)2 * (l + 1) * c.N);
    key_wsum(c, gk.keys.at(elt), KW, l);
    gk.kw[{elt, l}] = KW;
    return KW;
}

// the MAC-form key table of a Galois key (built on first use, see mac_key_table)
const u64 *galois_mkey(hec_context *ctx, hec_galois_keys &gk, u32 elt)
{
    auto it = gk.mkey.find(elt);
    if (it != gk.mkey.end()) return it->second;
    Ctx &c = ctx->c;
    u64 *MK = dalloc((std::size_t)c.L * 2 * c.K * c.N);
    mac_key_table(c, gk.keys.at(elt), MK, (u32)invm(elt, 2 * c.N));
    gk.mkey[elt] = MK;
    return MK;
}

// X (size 2) -> OUT = apply_galois(X, elt) followed by key switching (SEAL apply_galois_inplace).
// When OUT does not alias X the permutation is applied inside the key switch's loads (the INTT of c1,
// the target reuse in the MAC, the c0 add in the mod-down) and never materialised; otherwise X is
// first permuted into scratch.
void galois_ks(Ctx &c, Scratch &s, PolyArr X, PolyArr OUT, int B, int l, u32 elt, const u64 *key)
{
    const u64 N = c.N;
    const bool alias = OUT.p == X.p || !c.fuse_galois;
    if (!alias) {
        keyswitch(c, s, PolyArr{X.p + X.sk, X.sb, 0}, key, PolyArr{X.p, X.sb, X.sk}, 1, OUT, B, l, elt);
        return;
    }
    const std::size_t top = s.top;
    u64 *S = s.take((u64)2 * B * l * N);
    {
        ProfScope ps(c, "galois");
        galois_permute(c, X, PolyArr{S, l * N, (u64)B * l * N}, B, 2, l, elt);
    }
    keyswitch(c, s, PolyArr{S + (u64)B * l * N, l * N, 0}, key, PolyArr{S, l * N, 0}, 1, OUT, B, l);
    s.top = top;
}

// divide-and-round by q_{l-1}: X = B entries of nk polys at level l -> OUT at level l-1
void rescale_batch(Ctx &c, Scratch &s, PolyArr X, int B, int nk, int l, PolyArr OUT)
{
    ProfScope ps(c, "rescale");
    const u64 N = c.N;
    const std::size_t top = s.top;
    u64 *Y = s.take((u64)B * nk * N), *Z = s.take((u64)B * nk * (l - 1) * N);
    const int pm[1] = {l - 1};
    for (int k = 0; k < nk; ++k)
        ntt_strided(c, true, X.p + k * X.sk + (u64)(l - 1) * N, X.sb, Y + k * N, nk * N, 1, pm, B);
    divide_round(c, Y, nk * N, N, X, PolyArr{}, 0, OUT, B, nk, l - 1, l - 1, c.ql_inv[l].data(),
                 c.ql_inv_q[l].data(), Z);
    s.top = top;
}
std::size_t rescale_words(const Ctx &c, std::size_t B, std::size_t nk, std::size_t l)
{
    return c.N * B * nk * (1 + 2 * l) + 3 * 64;
}

void check_ct(const hec_context *ctx, const hec_ciphertext *a)
{
    need(a && a->ctx == ctx, "encrypted is not valid for encryption parameters");
    need(a->level >= 1 && a->level <= ctx->c.L && a->size >= 2 && a->d,
         "encrypted is not valid for encryption parameters");
}
void set_device(hec_context *ctx)
{
    need(ctx != nullptr, "context is null");
    HEC_HIP(hipSetDevice(ctx->c.device));
}

void d2d(Ctx &c, void *dst, const void *src, std::size_t words)
{
    if (!words) return;
    if (c.kernel_memops) dev_copy64(c, (u64 *)dst, (const u64 *)src, words);
    else HEC_HIP(hipMemcpyAsync(dst, src, words * sizeof(u64), hipMemcpyDeviceToDevice, c.stream));
}

// ------------------------------------------------------------------ he::linalg driver -----
struct MatvecPlan {
    std::size_t l = 0;
    double prod_scale = 0;
    std::vector<std::vector<u32>> elts;  // per diagonal j
};

// Rotation prefix trie.  SEAL's rotate_internal turns rot(x, j) into a fixed sequence of key
// switches (one per NAF term, least significant first).  Rotations of the SAME input by different
// j share prefixes of that sequence (rot by 5 = KS_4(KS_1(x)) starts with rot by 1), so a
// depth-first walk over the trie of sequences computes every distinct prefix once: each rot(x, j)
// is still produced by exactly SEAL's sequence of key switches applied to exactly the same
// intermediate ciphertexts, so the bits are unchanged (cfg3: 18,204 -> 5,460 key switches).
struct RotTrie {
    struct Node {
        u32 elt = 0;
        std::vector<int> children;
        std::vector<std::size_t> terminals;  // rotation amounts ending at this node
    };
    std::vector<Node> nodes{Node{}};
    int depth = 0;
    void insert(const std::vector<u32> &seq, std::size_t tag)
    {
        int cur = 0;
        for (u32 e : seq) {
            int nxt = -1;
            for (int c : nodes[cur].children)
                if (nodes[c].elt == e) { nxt = c; break; }
            if (nxt < 0) {
                nodes.push_back(Node{e, {}, {}});
                nxt = (int)nodes.size() - 1;
                nodes[cur].children.push_back(nxt);
            }
            cur = nxt;
        }
        nodes[cur].terminals.push_back(tag);
        depth = std::max(depth, (int)seq.size());
    }
    std::size_t key_switches() const { return nodes.size() - 1; }
};

// Rotation buffers of the trie walk: nb per depth, taken round robin by consecutive children at a
// depth, so the buffer of a visited terminal stays intact for nb - 1 more siblings (deferred tensors).
struct TrieBufs {
    std::vector<std::vector<u64 *>> b;  // [depth][slot]
    std::vector<unsigned> next;
    TrieBufs(Scratch &s, int depth, int nb, u64 words) : b(depth + 1), next(depth + 1, 0)
    {
        for (int d = 0; d <= depth; ++d)
            for (int k = 0; k < (d == 0 ? 1 : nb); ++k) b[d].push_back(s.take(words));
    }
    u64 *take(int d) { return b[d][next[d]++ % b[d].size()]; }
};

// Depth-first walk: visit(tag, src) for every terminal of `node`, then for each child compute the
// child's rotation into a depth + 1 buffer and recurse.  before_write(buf) runs before a buffer is
// overwritten (the caller flushes deferred work that still reads it).  A buffer is only rewritten
// after the subtree that read it has been enqueued (stream order makes that safe).
template <class F, class W>
void walk_trie(Ctx &c, Scratch &s, const RotTrie &t, int node, PolyArr src, int depth, int B, int l,
               const hec_galois_keys &gk, TrieBufs &bufs, u64 stride, F &visit, W &before_write)
{
    for (std::size_t tag : t.nodes[node].terminals) visit(tag, src);
    for (int ch : t.nodes[node].children) {
        const u32 e = t.nodes[ch].elt;
        const PolyArr dst{bufs.take(depth + 1), stride, (u64)l * c.N};
        before_write(dst.p);
        galois_ks(c, s, src, dst, B, l, e, gk.keys.at(e));
        walk_trie(c, s, t, ch, dst, depth + 1, B, l, gk, bufs, stride, visit, before_write);
    }
}

// The same walk with the hoisted mod-up (hec_kernels.hip): a node with at least min_children children
// computes INTT(c1) and the NTT-form digits of every (target prime, digit) once into hs[depth]; each
// child then only runs the hoisted key MAC and the mod-down.  Nodes with fewer children use the fused
// per-rotation key switch.
template <class F, class W>
void walk_trie_hoisted(Ctx &c, Scratch &s, const RotTrie &t, int node, PolyArr src, int depth, int B, int l,
                       hec_context *ctx, hec_galois_keys &gk, TrieBufs &bufs, const std::vector<Hoist> &hs,
                       u64 stride, int min_children, F &visit, W &before_write)
{
    for (std::size_t tag : t.nodes[node].terminals) visit(tag, src);
    const auto &ch = t.nodes[node].children;
    if ((int)ch.size() < min_children) {
        for (int cn : ch) {
            const u32 e = t.nodes[cn].elt;
            const PolyArr dst{bufs.take(depth + 1), stride, (u64)l * c.N};
            before_write(dst.p);
            galois_ks(c, s, src, dst, B, l, e, gk.keys.at(e));
            walk_trie_hoisted(c, s, t, cn, dst, depth + 1, B, l, ctx, gk, bufs, hs, stride, min_children, visit,
                              before_write);
        }
        return;
    }
    const Hoist &h = hs[depth];
    hoist_node(c, src, B, l, h);
    if (c.debug_lanes) debug_count_zl(c, h.zl, c.zflag + 1);
    const u64 N = c.N;
    // children in groups of up to `sup` siblings: one sibling-fused k_hmacm launch per hoisted_group() of them (the
    // default hmac_cfg 2: the whole group, slots of 2; 1: per pair), accumulators h.acc(q), contiguous; then the
    // mod-downs in groups of HOIST_GROUP share their small launches
    const std::size_t grp = (std::size_t)hoisted_group(c);
    const std::size_t sup = std::max<std::size_t>(grp, HOIST_GROUP / grp * grp);
    // the sibling-fused MAC folds the node's c0 into the children's accumulators (X0 P mod q_I), so their
    // mod-downs take no IN term; the one-child MAC (hmac_cfg 0) does not
    const bool fold = c.hmac_cfg != 0;
    const PolyArr X0 = fold ? PolyArr{src.p, src.sb, src.sk} : PolyArr{};
    const int in_nk = fold ? 0 : 1;
    for (std::size_t g0 = 0; g0 < ch.size(); g0 += sup) {
        const int ng = (int)std::min<std::size_t>(sup, ch.size() - g0);
        HChildSpec kids[HOIST_GROUP];
        for (int q = 0; q < ng; ++q) {
            const u32 e = t.nodes[ch[g0 + q]].elt;
            kids[q] = HChildSpec{e, (u32)invm(e, 2 * N), gk.keys.at(e), galois_negw(ctx, gk, e), h.acc(q),
                                 galois_kw(ctx, gk, e, l), fold ? galois_mkey(ctx, gk, e) : nullptr};
        }
        const double K = l + 1;  // per child: key (2 l K), W (K), KW (2 K), ACC (2 B K)
        for (int q0 = 0, nk = 0; q0 < ng; q0 += nk) {  // one profile scope per launch (bench.py's roofline)
            nk = std::min((int)grp, ng - q0);
            // an odd group's last three children as one 3-child launch (the digits read once, not twice)
            if (c.hmac_odd3 && grp == 2 && ng - q0 == 3) nk = 3;
            ProfScope ps(c, "ks_hmac");  // digits E (B l^2) + c1 (B l) [+ c0 (B l), folded] + per child
            ProfScope k(c, "k:k_hmacm",
                        (double)B * (l * l + l + (fold ? l : 0)) + nk * (2.0 * l * K + 3.0 * K + 2.0 * B * K));
            if (c.hmac_cfg == 2)
                hoisted_mac_group(c, PolyArr{src.p + src.sk, src.sb, 0}, X0, h.E, h.zl, kids + q0, nk, B, l);
            else if (nk == 3 && grp == 2)
                hoisted_mac_3(c, PolyArr{src.p + src.sk, src.sb, 0}, X0, h.E, h.zl, kids + q0, B, l);
            else hoisted_mac_multi(c, PolyArr{src.p + src.sk, src.sb, 0}, X0, h.E, h.zl, kids + q0, nk, B, l);
        }
        for (int m0 = 0; m0 < ng; m0 += HOIST_GROUP) {  // mod-downs in groups, then each child's subtree
            const int nm = std::min(HOIST_GROUP, ng - m0);
            if ((int)bufs.b[depth + 1].size() < nm) {  // too few rotation buffers to hold the group at once
                for (int q = m0; q < m0 + nm; ++q) {
                    const PolyArr dst{bufs.take(depth + 1), stride, (u64)l * N};
                    before_write(dst.p);
                    const std::size_t top = s.top;
                    u64 *Z = s.take((u64)B * 2 * l * N);
                    moddown(c, h.acc(q), Z, PolyArr{src.p, src.sb, src.sk}, in_nk, dst, B, l, kids[q].elt);
                    s.top = top;
                    walk_trie_hoisted(c, s, t, ch[g0 + q], dst, depth + 1, B, l, ctx, gk, bufs, hs, stride,
                                      min_children, visit, before_write);
                }
                continue;
            }
            PolyArr dst[HOIST_GROUP];
            u32 elts[HOIST_GROUP];
            for (int q = 0; q < nm; ++q) {
                dst[q] = PolyArr{bufs.take(depth + 1), stride, (u64)l * N};
                before_write(dst[q].p);
                elts[q] = kids[m0 + q].elt;
            }
            {
                const std::size_t top = s.top;
                u64 *Z = s.take((u64)nm * B * 2 * l * N);
                moddown_group(c, h.acc(m0), Z, PolyArr{src.p, src.sb, src.sk}, in_nk, dst, elts, nm, B, l);
                s.top = top;
            }
            for (int q = 0; q < nm; ++q)
                walk_trie_hoisted(c, s, t, ch[g0 + m0 + q], dst[q], depth + 1, B, l, ctx, gk, bufs, hs, stride,
                                  min_children, visit, before_write);
        }
    }
}

// The argument checks SEAL runs along the reference loop (rotate_internal, multiply[_plain]_inplace's
// scale bound, add_inplace's are_close, relinearize / rescale at the end of the chain), in its order, on
// the host.  Returns the product scale of every output.  matvec_lanes runs it on the calling thread over
// the whole batch before any lane starts, so a failing call writes no output (as in SEAL).
std::vector<double> matvec_check(hec_context *ctx, const hec_ciphertext *const *diags, const hec_plaintext *const *pdiags,
                                 std::size_t n, const std::vector<std::size_t> &js, const hec_ciphertext *const *cols,
                                 std::size_t p, const hec_kswitch_key *rk, const hec_galois_keys *gk, bool finish)
{
    const Ctx &c = ctx->c;
    const bool pt = pdiags != nullptr;
    need(n >= 1 && p >= 1 && !js.empty(), "empty matrix operand");
    for (std::size_t j : js) need(j < n, "diagonal index out of range");
    need(gk && gk->ctx == ctx, "galois_keys is not valid for encryption parameters");
    if (finish && !pt) need(rk && rk->ctx == ctx, "relin_keys is not valid for encryption parameters");
    const std::size_t l = cols[0]->level;
    for (std::size_t i = 0; i < p; ++i) check_ct(ctx, cols[i]);
    for (std::size_t i = 0; i < p; ++i) need(cols[i]->size == 2, "encrypted size must be 2");
    for (std::size_t i = 0; i < p; ++i) need(cols[i]->level == l, "encrypted1 and encrypted2 parameter mismatch");
    if (pt) {
        for (std::size_t j : js)
            need(pdiags[j] && pdiags[j]->ctx == ctx && pdiags[j]->d, "plain is not valid for encryption parameters");
        for (std::size_t j : js) need(pdiags[j]->level == l, "encrypted_ntt and plain_ntt parameter mismatch");
    } else {
        for (std::size_t j : js) check_ct(ctx, diags[j]);
        for (std::size_t j : js) need(diags[j]->size == 2, "encrypted size must be 2");
        for (std::size_t j : js) need(diags[j]->level == l, "encrypted1 and encrypted2 parameter mismatch");
    }
    auto dscale = [&](std::size_t j) { return pt ? pdiags[j]->scale : diags[j]->scale; };
    // scale bookkeeping exactly as multiply[_plain]_inplace (bound) + add_inplace (are_close) would see it
    std::vector<double> ps(p);
    for (std::size_t i = 0; i < p; ++i) {
        for (std::size_t k = 0; k < js.size(); ++k) {
            const double sc = cols[i]->scale * dscale(js[k]);
            need(scale_ok(c, sc, l), "scale out of bounds");
            if (k == 0) ps[i] = sc;
            else need(are_close(ps[i], sc), "scale mismatch");
        }
    }
    if (finish && l < 2) throw std::invalid_argument("end of modulus switching chain reached");
    std::vector<u32> seq;  // rotate_internal's own errors ("step count too large", "Galois key not present")
    for (std::size_t j : js) {
        seq.clear();
        rotation_elts(c, (int)j, *gk, seq);
    }
    return ps;
}

// BatchedMatrix::matmul diag x col (he_linalg.cpp:943-1006) for the p columns at once, diagonals
// [jb, je).  The loop over i (output column) is interchanged with the loop over j so that one
// rotation launch sequence and one key read serve all p columns, and the rotations run over the
// prefix trie; every out[i] still sums the same terms (modular addition is exact and order free),
// so the bits equal the reference loop's.
// diags (ciphertexts) or pdiags (plaintexts, the ct x pt form: multiply_plain, products stay size 2,
// no relinearization) — exactly one is non-null.
void matvec_core(hec_context *ctx, const hec_ciphertext *const *diags, const hec_plaintext *const *pdiags,
                 std::size_t n, const std::vector<std::size_t> &js, const hec_ciphertext *const *cols, std::size_t p,
                 const hec_kswitch_key *rk, const hec_galois_keys *gk, bool finish, hec_ciphertext *const *out,
                 Ctx *exec = nullptr)  // exec: the lane context that runs it (objects still belong to ctx)
{
    Ctx &c = exec ? *exec : ctx->c;
    const bool pt = pdiags != nullptr;
    const std::vector<double> ps = matvec_check(ctx, diags, pdiags, n, js, cols, p, rk, gk, finish);
    const std::size_t l = cols[0]->level, N = c.N;
    auto ddata = [&](std::size_t j) -> const u64 * { return pt ? pdiags[j]->d : diags[j]->d; };
    RotTrie trie;
    {
        std::vector<u32> seq;
        for (std::size_t j : js) {
            seq.clear();
            rotation_elts(c, (int)j, *gk, seq);
            trie.insert(seq, j);
        }
    }
    const u64 S2 = 2 * l * N, S3 = 3 * l * N;
    const int D = trie.depth;
    const int nb = c.tensor_defer_bufs;  // rotation buffers per depth
    const bool hoist = c.hoist && D > 0;
    std::size_t words = p * (S2 * (1 + (std::size_t)D * nb) + S3) + 2 * p * l * N + ks_words(c, p, l) +
                        (D * nb + 80) * 64;
    if (hoist) {
        words += (std::size_t)D * hoist_words(c, p, l);
        words += hoisted_child_words(c, p, l);
    }
    if (finish) words += rescale_words(c, p, 2, l) + p * 2 * (l - 1) * N;
    Scratch s(c, words);
    TrieBufs bufs(s, D, nb, p * S2);
    u64 *ACC3 = s.take(p * S3);
    for (std::size_t i = 0; i < p; ++i) d2d(c, bufs.b[0][0] + i * S2, cols[i]->d, S2);
    const PolyArr Xa{bufs.b[0][0], S2, l * N}, Aa{ACC3, S3, l * N};
    bool first = true;
    // the products of up to TB_MAX visited terminals (ct x ct tensors, or ct x pt plain products) are
    // deferred and applied in one k_tensor_multi pass (the accumulator read/written once per batch); a
    // batch is flushed when full or before one of its rotation buffers is overwritten
    TensorBatch tb{};
    auto flush = [&] {
        if (tb.T == 0) return;
        ProfScope pr(c, "tensor");
        // T rotated inputs (2 B l each) + T diagonals (2 l, or l plaintext) + ACC read (unless first) + write
        const double accl = (pt ? 2.0 : 3.0) * p * l;
        ProfScope k(c, "k:k_tensor_multi2", tb.T * (2.0 * p * l + (pt ? 1.0 : 2.0) * l) + (first ? 1 : 2) * accl);
        tensor_multi(c, tb, S2, l * N, l * N, Aa, (int)p, (int)l, first, pt);
        first = false;
        tb.T = 0;
    };
    auto visit = [&](std::size_t j, PolyArr src) {
        tb.r[tb.T] = src.p;
        tb.a[tb.T] = ddata(j);
        if (++tb.T == std::min(TB_MAX, c.tensor_defer_max)) flush();
    };
    auto before_write = [&](const u64 *buf) {
        for (int t = 0; t < tb.T; ++t)
            if (tb.r[t] == buf) return flush();
    };
    if (hoist) {
        hec_galois_keys &gkm = const_cast<hec_galois_keys &>(*gk);  // negw is a per-key cache
        for (std::size_t nd = 1; nd < trie.nodes.size(); ++nd) {
            galois_negw(ctx, gkm, trie.nodes[nd].elt);
            galois_kw(ctx, gkm, trie.nodes[nd].elt, (int)l);
            if (c.hmac_cfg != 0) galois_mkey(ctx, gkm, trie.nodes[nd].elt);
        }
        std::vector<Hoist> hs(D);
        for (int d = 0; d < D; ++d) hs[d] = hoist_alloc(c, s, (int)p, (int)l);
        dev_zero(c, c.zflag, 2 * sizeof(int));
        walk_trie_hoisted(c, s, trie, 0, Xa, 0, (int)p, (int)l, ctx, gkm, bufs, hs, S2, c.hoist_min_children, visit,
                          before_write);
    } else {
        walk_trie(c, s, trie, 0, Xa, 0, (int)p, (int)l, *gk, bufs, S2, visit, before_write);
    }
    flush();
    if (hoist) {  // a digit limb with more zero coefficients than the hoisted MAC corrects: recompute
        int zfl[2] = {0, 0};
        HEC_HIP(hipMemcpyAsync(zfl, c.zflag, 2 * sizeof(int), hipMemcpyDeviceToHost, c.stream));
        HEC_HIP(hipStreamSynchronize(c.stream));
        const int zf = zfl[0];
        if (c.debug_lanes)
            std::fprintf(stderr, "hec-debug: %s p=%zu zero-list nodes %d overflow %d\n", exec ? "lane" : "ctx", p, zfl[1],
                         zfl[0]);
        if (zf) {
            if (std::getenv("HEC_DEBUG")) std::fprintf(stderr, "hec: zero-list overflow, matvec recomputed without hoisting (p=%zu)\n", p);
            c.hoist = false;
            try {
                matvec_core(ctx, diags, pdiags, n, js, cols, p, rk, gk, finish, out, exec);
            } catch (...) {
                c.hoist = true;
                throw;
            }
            c.hoist = true;
            return;
        }
    }
    const u64 accw = pt ? S2 : S3;  // accumulator words per output
    if (!finish) {
        for (std::size_t i = 0; i < p; ++i) {
            ensure(out[i], accw);
            d2d(c, out[i]->d, ACC3 + i * S3, accw);
            out[i]->size = pt ? 2 : 3; out[i]->level = l; out[i]->scale = ps[i];
        }
        return;
    }
    if (!pt) {  // relinearize (SMART_RELIN == 1: once per output) — he_linalg.cpp:1000
        ProfScope pr(c, "relin");
        keyswitch(c, s, PolyArr{ACC3 + 2 * l * N, S3, 0}, rk->d, Aa, 2, Aa, (int)p, (int)l);
    }
    const u64 So = 2 * (l - 1) * N;  // rescale (he_linalg.cpp:1001)
    u64 *O = s.take(p * So);
    rescale_batch(c, s, Aa, (int)p, 2, (int)l, PolyArr{O, So, (l - 1) * N});
    const double ql = (double)c.q[l - 1];
    for (std::size_t i = 0; i < p; ++i) {
        ensure(out[i], So);
        d2d(c, out[i]->d, O + i * So, So);
        out[i]->size = 2; out[i]->level = l - 1; out[i]->scale = ps[i] / ql;
    }
}


// ---------------------------------------------------------------- batch lanes
// The engine's kernels leave issue slots and bandwidth idle (they wait on memory for most of their
// cycles), so the batch of a matvec is split into up to c.lanes sub-batches of at least
// c.lane_min_batch vectors that run the same trie walk concurrently, each from its own host thread on its
// own HIP stream and workspace.  Outputs are independent per input vector, so the bits are unchanged.
hec_context *make_lane(hec_context *parent)
{
    auto *l = new hec_context();
    Ctx &c = l->c;
    c = parent->c;  // shared device tables (twiddles, primes, maps), host constants and knobs
    c.ws = Workspace{};
    c.ws.defer_free = true;  // grown from the lane's thread while the other lanes launch
    c.prof_mode = 0;
    c.prof_tab.clear();
    c.prof_pend.clear();
    c.ev_pool.clear();
    c.ev_used = 0;
    c.stream = nullptr;
    c.zflag = nullptr;
    HEC_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    c.own_stream = true;
    HEC_HIP(hipMalloc(&c.zflag, 2 * sizeof(int)));
    HEC_HIP(hipMemset(c.zflag, 0, 2 * sizeof(int)));
    HEC_HIP(hipEventCreateWithFlags(&l->lane_done, hipEventDisableTiming));
    return l;
}
void free_lane(hec_context *l)
{
    Ctx &c = l->c;
    (void)hipStreamSynchronize(c.stream);
    if (l->lane_done) (void)hipEventDestroy(l->lane_done);
    c.ws.release();
    (void)hipFree(c.zflag);
    (void)hipStreamDestroy(c.stream);
    delete l;
}

// HEC_DEBUG_LANES: a checksum of every key's sign-mask NTTs W and key sums KW at this level, compared with the first one
// seen (they are built once and must never change)
// first-seen checksums of the per-key tables, keyed by (key set, Galois element, level, table) -- not by device
// address, which a freed table hands on to another key set; a key set's entries leave with it
// (debug_key_tables_forget from hec_galois_keys_destroy)
static std::mutex g_dbg_mu;
static std::map<std::tuple<const hec_galois_keys *, u32, int, int>, u64> g_dbg_first;

static void debug_key_tables_forget(const hec_galois_keys *gk)
{
    std::lock_guard<std::mutex> lock(g_dbg_mu);
    for (auto it = g_dbg_first.begin(); it != g_dbg_first.end();)
        it = std::get<0>(it->first) == gk ? g_dbg_first.erase(it) : std::next(it);
}

void debug_key_tables(hec_context *ctx, const hec_galois_keys &gk, int l)
{
    std::lock_guard<std::mutex> lock(g_dbg_mu);
    Ctx &c = ctx->c;
    HEC_HIP(hipDeviceSynchronize());
    auto sum = [&](const u64 *d, std::size_t words) {
        std::vector<u64> h(words);
        HEC_HIP(hipMemcpy(h.data(), d, words * sizeof(u64), hipMemcpyDeviceToHost));
        u64 s = 1469598103934665603ull;
        for (u64 w : h) s = (s ^ w) * 1099511628211ull;
        return s;
    };
    int changed = 0, n = 0;
    for (const auto &kv : gk.negw) {
        const u64 sw = sum(kv.second, c.K * c.N);
        auto it = gk.kw.find({kv.first, l});
        const bool has_kw = it != gk.kw.end();
        const u64 sk = has_kw ? sum(it->second, (std::size_t)2 * (l + 1) * c.N) : 0;
        for (auto [key, v] : {std::pair{std::tuple{&gk, (u32)kv.first, 0, 0}, sw},
                              std::pair{std::tuple{&gk, (u32)kv.first, l, 1}, sk}}) {
            if (std::get<3>(key) == 1 && !has_kw) continue;
            auto f = g_dbg_first.find(key);
            if (f == g_dbg_first.end()) g_dbg_first[key] = v;
            else if (f->second != v) ++changed;
            ++n;
        }
    }
    std::fprintf(stderr, "hec-debug: key tables %d checked, %d changed\n", n, changed);
}

void matvec_lanes(hec_context *ctx, const hec_ciphertext *const *diags, const hec_plaintext *const *pdiags,
                  std::size_t n, const std::vector<std::size_t> &js, const hec_ciphertext *const *cols, std::size_t p,
                  const hec_kswitch_key *rk, const hec_galois_keys *gk, bool finish, hec_ciphertext *const *out)
{
    Ctx &c = ctx->c;
    const int nl = (int)std::min<std::size_t>((std::size_t)std::max(1, c.lanes), p / std::max(1, c.lane_min_batch));
    if (nl <= 1 || c.prof_mode != 0) {  // profiling: the single-stream schedule, one phase at a time
        // a whole batch on the context's own workspace: first return the idle lanes' workspaces (at the bench's
        // 192 vectors the lanes hold 3 x 64 vectors' worth, and the one-lane profile step needs as much again)
        if (p > (std::size_t)std::max(1, c.lane_min_batch))
            for (hec_context *l : ctx->lanes) {
                HEC_HIP(hipStreamSynchronize(l->c.stream));
                l->c.ws.release();
            }
        matvec_core(ctx, diags, pdiags, n, js, cols, p, rk, gk, finish, out);
        return;
    }
    matvec_check(ctx, diags, pdiags, n, js, cols, p, rk, gk, finish);  // whole batch, before any lane writes
    if (c.hoist) {  // the lazily built per-key tables, before the lanes only read them
        auto &gkm = const_cast<hec_galois_keys &>(*gk);
        for (auto &kv : gkm.keys) {
            galois_negw(ctx, gkm, kv.first);
            galois_kw(ctx, gkm, kv.first, (int)cols[0]->level);
            if (c.hmac_cfg != 0) galois_mkey(ctx, gkm, kv.first);
        }
    }
    // the outputs are sized here, on the calling thread, so no lane thread frees or allocates them (matvec_core's
    // ensure() then finds them large enough)
    {
        const std::size_t l = cols[0]->level, N = c.N;
        const std::size_t w = finish ? 2 * (l - 1) * N : (pdiags ? 2 : 3) * l * N;
        for (std::size_t i = 0; i < p; ++i) {
            need(out[i] != nullptr, "null argument");
            ensure(out[i], w);
        }
    }
    while ((int)ctx->lanes.size() < nl) ctx->lanes.push_back(make_lane(ctx));
    if (!ctx->lanes_start) HEC_HIP(hipEventCreateWithFlags(&ctx->lanes_start, hipEventDisableTiming));
    hipEvent_t start = ctx->lanes_start;
    HEC_HIP(hipEventRecord(start, c.stream));  // the inputs were produced on the context's stream
    std::vector<char> done(nl, 0);
    std::vector<std::exception_ptr> err(nl);
    std::vector<std::thread> th;
    for (int i = 0; i < nl; ++i) {
        const std::size_t b0 = p * i / nl, b1 = p * (i + 1) / nl;
        th.emplace_back([&, i, b0, b1] {
            try {
                Ctx &lc = ctx->lanes[i]->c;
                HEC_HIP(hipSetDevice(lc.device));
                HEC_HIP(hipStreamWaitEvent(lc.stream, start, 0));
                matvec_core(ctx, diags, pdiags, n, js, cols + b0, b1 - b0, rk, gk, finish, out + b0, &lc);
                HEC_HIP(hipEventRecord(ctx->lanes[i]->lane_done, lc.stream));
                if (c.lane_serial) HEC_HIP(hipStreamSynchronize(lc.stream));
                done[i] = 1;
            } catch (...) {
                err[i] = std::current_exception();
            }
        });
        if (c.lane_serial) th.back().join();
    }
    for (auto &t : th)
        if (t.joinable()) t.join();
    for (int i = 0; i < nl; ++i)  // later work on the context sees the outputs
        if (done[i]) HEC_HIP(hipStreamWaitEvent(c.stream, ctx->lanes[i]->lane_done, 0));
    for (int i = 0; i < nl; ++i)  // outgrown lane workspaces, now that no lane thread runs (waits only after a growth)
        ctx->lanes[i]->c.ws.reclaim(ctx->lanes[i]->c.stream);
    if (c.debug_lanes && c.hoist) debug_key_tables(ctx, *gk, (int)cols[0]->level);
    for (auto &e : err)
        if (e) std::rethrow_exception(e);
}

// ---------------------------------------------------------------- multi-GPU planner and RCCL
// The diagonal planner: SEAL's key-switch sequence of every rotation j < n (rotate_internal over the key
// set), the diagonals ordered depth-first over the rotation prefix trie (lexicographic order of the
// sequences keeps every subtree contiguous), then cut into `world` chunks with the smallest key-switch
// budget per chunk that fits (binary search).  A cut inside a subtree only repeats the path above it, so
// the ranks together spend about the 1-GPU trie's key switches.  Same rule as shard.plan_diagonal_shards.
void plan_elts(std::size_t N, int step, const std::set<u32> &keys, std::vector<u32> &out)
{
    if (step == 0) return;
    const u64 m = 2 * N;
    const u64 s = step < 0 ? (u64)((long)N / 2 + step) : (u64)step;
    u64 e = 1;
    for (u64 k = 0; k < s; ++k) e = e * 3 % m;
    if (keys.count((u32)e)) { out.push_back((u32)e); return; }
    for (int t : naf(step))
        if ((std::size_t)std::abs(t) != N / 2) plan_elts(N, t, keys, out);
}
std::vector<std::vector<std::size_t>> plan_shards(std::size_t N, std::size_t n, int world, const std::set<u32> &keys)
{
    need(world >= 1 && (std::size_t)world <= n, "need 1 <= world <= n");
    std::vector<std::vector<u32>> seq(n);
    for (std::size_t j = 0; j < n; ++j) plan_elts(N, (int)j, keys, seq[j]);
    std::vector<std::size_t> order(n);
    for (std::size_t j = 0; j < n; ++j) order[j] = j;
    std::stable_sort(order.begin(), order.end(), [&](std::size_t a, std::size_t b) { return seq[a] < seq[b]; });
    auto prefixes = [&](std::size_t j) {
        std::vector<std::vector<u32>> pre;
        for (std::size_t k = 1; k <= seq[j].size(); ++k) pre.emplace_back(seq[j].begin(), seq[j].begin() + k);
        return pre;
    };
    std::set<std::vector<u32>> all;
    for (std::size_t j = 0; j < n; ++j)
        for (auto &x : prefixes(j)) all.insert(x);
    const std::size_t total = all.size();
    auto chunk = [&](std::size_t budget, std::size_t limit, std::vector<std::vector<std::size_t>> &out) {
        out.clear();
        std::vector<std::size_t> cur;
        std::set<std::vector<u32>> seen;
        std::size_t cost = 0;
        for (std::size_t j : order) {
            const auto pre = prefixes(j);
            std::size_t add = 0;
            for (auto &x : pre) add += seen.count(x) ? 0 : 1;
            if (!cur.empty() && cost + add > budget) {
                out.push_back(cur);
                if (out.size() >= limit) return false;
                cur.clear();
                seen.clear();
                cost = 0;
                add = pre.size();
            }
            cur.push_back(j);
            for (auto &x : pre) seen.insert(x);
            cost += add;
        }
        out.push_back(cur);
        return true;
    };
    std::size_t lo = std::max<std::size_t>(1, total / (std::size_t)world), hi = total + 1;
    std::vector<std::vector<std::size_t>> best, tmp;
    while (lo <= hi) {
        const std::size_t mid = (lo + hi) / 2;
        if (chunk(mid, (std::size_t)world, tmp)) {
            best = tmp;
            hi = mid - 1;
        } else {
            lo = mid + 1;
        }
    }
    while ((int)best.size() < world) {  // split the largest chunks until every rank has one
        std::size_t k = 0;
        for (std::size_t i = 1; i < best.size(); ++i)
            if (best[i].size() > best[k].size()) k = i;
        std::vector<std::size_t> c = best[k];
        best.erase(best.begin() + (long)k);
        best.insert(best.begin() + (long)k, std::vector<std::size_t>(c.begin() + (long)(c.size() / 2), c.end()));
        best.insert(best.begin() + (long)k, std::vector<std::size_t>(c.begin(), c.begin() + (long)(c.size() / 2)));
    }
    for (auto &c : best) std::sort(c.begin(), c.end());
    return best;
}

// RCCL, loaded on first use (the engine itself does not link it): the functions of rccl.h we call
struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};
const Rccl &rccl()
{
    static Rccl r;
    static bool tried = false;
    static std::mutex mu;
    std::lock_guard<std::mutex> lock(mu);
    if (!tried) {
        tried = true;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (h) {
            r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
            r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
            r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
            r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
            r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        }
    }
    if (!r.get_unique_id || !r.init_rank || !r.all_reduce || !r.destroy)
        throw std::logic_error("RCCL (librccl.so.1) is not available");
    return r;
}
void nccl_check(ncclResult_t e, const char *what)
{
    if (e != ncclSuccess)
        throw std::logic_error(std::string(what) + ": " + (rccl().error_string ? rccl().error_string(e) : "RCCL error"));
}

struct RcclComm final : HecComm {
    ncclComm_t comm;
    explicit RcclComm(ncclComm_t c) : comm(c) {}
    ~RcclComm() override { (void)rccl().destroy(comm); }
    void allreduce_f64(double *host, std::size_t n, int op, hipStream_t s) override
    {
        double *dv = nullptr;
        HEC_HIP(hipMallocAsync((void **)&dv, n * sizeof(double), s));
        HEC_HIP(hipMemcpyAsync(dv, host, n * sizeof(double), hipMemcpyHostToDevice, s));
        nccl_check(rccl().all_reduce(dv, dv, n, ncclFloat64, op == HEC_REDUCE_MIN ? ncclMin : ncclMax, comm, s),
                   "ncclAllReduce");
        HEC_HIP(hipMemcpyAsync(host, dv, n * sizeof(double), hipMemcpyDeviceToHost, s));
        HEC_HIP(hipFreeAsync(dv, s));
        HEC_HIP(hipStreamSynchronize(s));
    }
    void allreduce_u64_sum(u64 *dev, std::size_t n, hipStream_t s) override
    {
        nccl_check(rccl().all_reduce(dev, dev, n, ncclUint64, ncclSum, comm, s), "ncclAllReduce");
    }
};

// the caller's host collectives (hec_comm_ops): MPI, torch.distributed (gloo), ...
struct OpsComm final : HecComm {
    hec_comm_ops ops;
    explicit OpsComm(const hec_comm_ops &o) : ops(o) {}
    void allreduce_f64(double *host, std::size_t n, int op, hipStream_t) override
    {
        if (ops.allreduce_f64(ops.user, host, n, op) != 0) throw std::logic_error("hec_comm_ops allreduce_f64 failed");
    }
    void allreduce_u64_sum(u64 *dev, std::size_t n, hipStream_t s) override
    {
        std::vector<u64> h(n);
        HEC_HIP(hipMemcpyAsync(h.data(), dev, n * sizeof(u64), hipMemcpyDeviceToHost, s));
        HEC_HIP(hipStreamSynchronize(s));
        if (ops.allreduce_u64_sum(ops.user, h.data(), n) != 0)
            throw std::logic_error("hec_comm_ops allreduce_u64_sum failed");
        HEC_HIP(hipMemcpyAsync(dev, h.data(), n * sizeof(u64), hipMemcpyHostToDevice, s));
        HEC_HIP(hipStreamSynchronize(s));
    }
};

// The sharded matvec's agreement step, before any data-path collective: every rank contributes its own argument
// check (status, SEAL's message) and its p product scales; all ranks return the same verdict, so an argument error
// on one rank is an error on every rank instead of a rank left waiting in the exchange, and SEAL's add_inplace "scale
// mismatch" is checked over the whole sum (he_linalg.cpp:977-997 adds every rank's terms).  Two all-reduces of p + 1
// doubles: [0] = (status << 8) | (rank + 1) of a failing rank (max, so the highest failing rank names the error),
// [1 .. p] the scales (min and max; a failing rank contributes +inf / -inf so it never decides the comparison).
int shard_agree(HecComm &cm, int rank, int status, std::string &msg, const double *ps, std::size_t p, hipStream_t s)
{
    std::vector<double> mn(1 + p), mx(1 + p);
    mn[0] = mx[0] = status ? (double)((status << 8) | (rank + 1)) : 0.0;
    for (std::size_t i = 0; i < p; ++i) {
        mn[1 + i] = status ? std::numeric_limits<double>::infinity() : ps[i];
        mx[1 + i] = status ? -std::numeric_limits<double>::infinity() : ps[i];
    }
    cm.allreduce_f64(mn.data(), mn.size(), HEC_REDUCE_MIN, s);
    cm.allreduce_f64(mx.data(), mx.size(), HEC_REDUCE_MAX, s);
    const int agreed = (int)mx[0];
    if (!status && agreed) {
        status = agreed >> 8;
        msg = "matmul_diag_col_sharded: the arguments failed SEAL's checks on rank " + std::to_string((agreed & 0xff) - 1);
    }
    if (!status)
        for (std::size_t i = 0; i < p; ++i)
            if (!are_close(mn[1 + i], mx[1 + i])) {
                status = HEC_EINVAL;
                msg = "scale mismatch";
                break;
            }
    return status;
}
}  // namespace

// =============================================================================== workspace ==
void hec::Workspace::reserve(std::size_t w, hipStream_t stream)
{
    if (w <= words) return;
    if (std::getenv("HEC_DEBUG")) std::fprintf(stderr, "hec: workspace %zu -> %zu words\n", words, w);
    (void)stream;
    if (base) retired.push_back(base);  // reclaimed later (see Workspace)
    base = dalloc(w);
    words = w;
}
void hec::Workspace::reclaim(hipStream_t stream)
{
    if (retired.empty()) return;
    HEC_HIP(hipStreamSynchronize(stream));
    for (u64 *p : retired) HEC_HIP(hipFree(p));
    retired.clear();
}
void hec::Workspace::release()
{
    if (base) (void)hipFree(base);
    for (u64 *p : retired) (void)hipFree(p);
    retired.clear();
    base = nullptr;
    words = 0;
}

// =============================================================================== C-ABI =====
extern "C" {

const char *hec_last_error(void) { return g_err.c_str(); }
int hec_version(void) { return 100; }

int hec_create_coeff_modulus(uint64_t N, const int *bit_sizes, uint64_t count, uint64_t *out)
{
    return guard([&] {
        need(N >= 2 && !(N & (N - 1)), "poly_modulus_degree is invalid");
        std::map<int, std::size_t> cnt;
        for (uint64_t i = 0; i < count; ++i) {
            need(bit_sizes[i] >= 2 && bit_sizes[i] <= 60, "bit_sizes is invalid");
            ++cnt[bit_sizes[i]];
        }
        const u64 factor = 2 * N;
        std::map<int, std::vector<u64>> table;
        for (auto &[b, k] : cnt) {  // SEAL util::get_primes: walk down from ((2^b-1)/2N)*2N+1
            u64 v = (((u64)1 << b) - 1) / factor * factor + 1;
            const u64 lo = (u64)1 << (b - 1);
            std::size_t left = k;
            while (left && v > lo) {
                if (isprime(v)) { table[b].push_back(v); --left; }
                v -= factor;
            }
            if (left) throw std::logic_error("failed to find enough qualifying primes");
        }
        for (uint64_t i = 0; i < count; ++i) {  // CoeffModulus::Create: back(), pop_back()
            out[i] = table[bit_sizes[i]].back();
            table[bit_sizes[i]].pop_back();
        }
    });
}

int hec_context_create(uint64_t N, const uint64_t *mod, uint64_t K, int device, hec_context **out)
{
    return guard([&] {
        need(out != nullptr, "out is null");
        need(N >= 1024 && N <= 65536 && !(N & (N - 1)), "poly_modulus_degree must be a power of two in [2^10, 2^16]");
        need(K >= 2 && K - 1 <= HEC_MAXL, "coeff_modulus size is invalid");
        // SEAL's context validation: every modulus at most SEAL_USER_MOD_BIT_COUNT_MAX = 60 bits, prime,
        // = 1 mod 2N (NTT-friendly) and pairwise coprime.  The 60-bit bound is also what keeps the sharded
        // exchange's plain int64 sum of up to 8 partial residues exact (shard.py exchange_partials).
        for (uint64_t i = 0; i < K; ++i)
            need(isprime(mod[i]) && (mod[i] - 1) % (2 * N) == 0 && !(mod[i] >> 60), "coeff_modulus is invalid");
        for (uint64_t i = 0; i < K; ++i)
            for (uint64_t j = 0; j < i; ++j) need(mod[i] != mod[j], "coeff_modulus is invalid");
        HEC_HIP(hipSetDevice(device));
        auto *ctx = new hec_context();
        Ctx &c = ctx->c;
        c.device = device;
        if (const char *f = std::getenv("HEC_FUSED_MODUP_MAC")) c.fused_modup_mac = f[0] != '0';
        if (const char *f = std::getenv("HEC_FUSE_GALOIS")) c.fuse_galois = f[0] != '0';
        if (const char *f = std::getenv("HEC_FAN")) c.fan_out = f[0] != '0';
        if (const char *f = std::getenv("HEC_HOIST_SCAN")) c.hoist_scan = std::atoi(f);
        if (const char *f = std::getenv("HEC_LANES")) c.lanes = std::max(1, std::atoi(f));
        if (const char *f = std::getenv("HEC_HOIST")) c.hoist = f[0] != '0';
        if (const char *f = std::getenv("HEC_HMAC")) c.hmac_cfg = std::atoi(f);
        if (const char *f = std::getenv("HEC_HMAC_ODD3")) c.hmac_odd3 = std::atoi(f);
        if (const char *f = std::getenv("HEC_HOIST_MIN")) c.hoist_min_children = std::max(1, std::atoi(f));
        if (const char *f = std::getenv("HEC_TENSOR_DEFER")) c.tensor_defer_max = std::max(1, std::atoi(f));
        if (const char *f = std::getenv("HEC_TENSOR_BUFS")) c.tensor_defer_bufs = std::max(1, std::atoi(f));
        if (const char *f = std::getenv("HEC_TENSOR_XCD")) c.tensor_xcd = std::max(0, std::atoi(f));
        if (const char *f = std::getenv("HEC_POISON")) c.poison = f[0] != '0';
        if (const char *f = std::getenv("HEC_LANE_SERIAL")) c.lane_serial = f[0] != '0';
        if (const char *f = std::getenv("HEC_DEBUG_LANES")) c.debug_lanes = f[0] != '0';
        if (const char *f = std::getenv("HEC_KERNEL_MEMOPS")) c.kernel_memops = f[0] != '0';
        if (const char *f = std::getenv("HEC_SPLIT_BFLY")) c.split_bfly = std::atoi(f);
        if (const char *f = std::getenv("HEC_NTTB_SHFL")) c.nttb_shfl = std::min(2, std::max(0, std::atoi(f)));
        if (const char *f = std::getenv("HEC_NTTB_SHFL_DR")) c.nttb_shfl_dr = std::atoi(f) != 0;
        if (const char *f = std::getenv("HEC_HMAC_INT")) c.hmac_int = std::atoi(f) != 0;
        if (const char *f = std::getenv("HEC_MODDOWN1")) c.moddown1 = std::atoi(f) != 0;
        if (const char *f = std::getenv("HEC_NT_E")) c.nt_e = std::atoi(f) != 0;
        if (const char *f = std::getenv("HEC_BMAC_SPLIT")) c.bmac_split = f[0] != '0';
        c.N = N;
        c.logN = __builtin_ctzll(N);
        c.K = K;
        c.L = K - 1;
        c.q.assign(mod, mod + K);
        for (u64 q : c.q) c.bits.push_back(64 - __builtin_clzll(q));
        HEC_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
        c.own_stream = true;
        std::vector<ulonglong2> tw(K * N), itw(K * N);
        std::vector<u64> psipow(K * 2 * N);  // hoisted mod-up: psi_i^e, e in [0, 2N)
        for (uint64_t i = 0; i < K; ++i) {
            const u64 q = c.q[i];
            DevPrime p{};
            p.q = q;
            u128 all = ~(u128)0, r = all / q;
            if (all % q == q - 1) r += 1;
            p.r0 = (u64)r;
            p.r1 = (u64)(r >> 64);
            p.ninv = invm(N % q, q);
            p.ninv_q = shoupq(p.ninv, q);
            p.fp = q < (1ull << 42) ? 1 : 0;  // exact FP64 NTT arithmetic (hec_device.h)
            p.qd = (double)q;
            p.qinv = 1.0 / (double)q;
            p.ninv_d = (double)p.ninv;
            c.hprimes.push_back(p);
            const u64 root = minimal_root(2 * N, q), iroot = invm(root, q);
            {
                u64 e = 1;
                for (uint64_t k = 0; k < 2 * N; ++k) {
                    psipow[i * 2 * N + k] = e;
                    e = (u64)((u128)e * root % q);
                }
            }
            u64 pw = 1, ipw = 1;
            for (uint64_t k = 0; k < N; ++k) {  // tw[bitrev(k)] = root^k
                const u32 t = brev((u32)k, c.logN);
                tw[i * N + t] = ulonglong2{pw, shoupq(pw, q)};
                itw[i * N + t] = ulonglong2{ipw, shoupq(ipw, q)};
                pw = (u64)((u128)pw * root % q);
                ipw = (u64)((u128)ipw * iroot % q);
            }
        }
        // pass-B re-laid tables: entry (s, i, r) = tw[(R + r) 2^s + i] at R (2^s - 1) + i R + r
        c.logR = (c.logN + 1) / 2;
        const uint64_t R = 1ull << c.logR, C = N / R;
        std::vector<ulonglong2> twb(K * N), itwb(K * N);
        for (uint64_t i = 0; i < K; ++i)
            for (uint64_t s = 0; (1ull << s) < C; ++s)
                for (uint64_t ii = 0; ii < (1ull << s); ++ii)
                    for (uint64_t r = 0; r < R; ++r) {
                        const uint64_t dst = i * N + R * ((1ull << s) - 1) + ii * R + r;
                        const uint64_t src = i * N + (R + r) * (1ull << s) + ii;
                        twb[dst] = tw[src];
                        itwb[dst] = itw[src];
                    }
        auto to_d = [](const std::vector<ulonglong2> &v) {
            std::vector<double> r(v.size());
            for (std::size_t k = 0; k < v.size(); ++k) r[k] = (double)v[k].x;  // exact when q < 2^42
            return r;
        };
        const std::vector<double> twf = to_d(tw), itwf = to_d(itw), twbf = to_d(twb), itwbf = to_d(itwb);
        for (auto [dst, src] : {std::pair{&c.twf, &twf}, std::pair{&c.itwf, &itwf}, std::pair{&c.twbf, &twbf},
                                std::pair{&c.itwbf, &itwbf}}) {
            HEC_HIP(hipMalloc(dst, K * N * sizeof(double)));
            HEC_HIP(hipMemcpy(*dst, src->data(), K * N * sizeof(double), hipMemcpyHostToDevice));
        }
        HEC_HIP(hipMalloc(&c.twb, K * N * sizeof(ulonglong2)));
        HEC_HIP(hipMalloc(&c.itwb, K * N * sizeof(ulonglong2)));
        HEC_HIP(hipMemcpy(c.twb, twb.data(), K * N * sizeof(ulonglong2), hipMemcpyHostToDevice));
        HEC_HIP(hipMemcpy(c.itwb, itwb.data(), K * N * sizeof(ulonglong2), hipMemcpyHostToDevice));
        {   // pass-B layout of the split-input Shoup words (k_bmac's integer targets): a = w 2^31 mod q of twb
            std::vector<u64> tba(K * N, 0);
            for (uint64_t i = 0; i < K; ++i)
                if (!c.hprimes[i].fp)
                    for (uint64_t k = 0; k < N; ++k) tba[i * N + k] = (u64)(((u128)twb[i * N + k].x << 31) % c.q[i]);
            HEC_HIP(hipMalloc(&c.twbs, K * N * sizeof(u64)));
            HEC_HIP(hipMemcpy(c.twbs, tba.data(), K * N * sizeof(u64), hipMemcpyHostToDevice));
        }
        {   // hoisted mod-up constants: psi powers per key prime, q_J mod q_I
            HEC_HIP(hipMalloc(&c.psipow, psipow.size() * sizeof(u64)));
            HEC_HIP(hipMemcpy(c.psipow, psipow.data(), psipow.size() * sizeof(u64), hipMemcpyHostToDevice));
            std::vector<u64> cji(c.L * K);
            for (std::size_t J = 0; J < c.L; ++J)
                for (std::size_t I = 0; I < K; ++I) cji[J * K + I] = c.q[J] % c.q[I];
            HEC_HIP(hipMalloc(&c.cji, cji.size() * sizeof(u64)));
            HEC_HIP(hipMemcpy(c.cji, cji.data(), cji.size() * sizeof(u64), hipMemcpyHostToDevice));
            HEC_HIP(hipMalloc(&c.zflag, 2 * sizeof(int)));
            HEC_HIP(hipMemset(c.zflag, 0, 2 * sizeof(int)));
        }
        {   // target-prime order tables per level (integer primes first)
            std::vector<int> tab((c.L + 1) * (HEC_MAXL + 2), 0);
            c.imap_nint.assign(c.L + 1, 0);
            for (std::size_t l = 1; l <= c.L; ++l) {
                int *t = tab.data() + l * (HEC_MAXL + 2), n = 0;
                for (int pass = 0; pass < 2; ++pass)
                    for (int I = 0; I <= (int)l; ++I) {
                        const int kI = I == (int)l ? (int)K - 1 : I;
                        const bool fp = c.hprimes[kI].fp != 0;
                        if ((pass == 0) != fp) t[n++] = I;
                    }
                for (int I = 0; I <= (int)l; ++I)
                    if (!c.hprimes[I == (int)l ? K - 1 : I].fp) ++c.imap_nint[l];
            }
            HEC_HIP(hipMalloc(&c.imap, tab.size() * sizeof(int)));
            HEC_HIP(hipMemcpy(c.imap, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice));
        }
        HEC_HIP(hipMalloc(&c.primes, K * sizeof(DevPrime)));
        HEC_HIP(hipMemcpy(c.primes, c.hprimes.data(), K * sizeof(DevPrime), hipMemcpyHostToDevice));
        HEC_HIP(hipMalloc(&c.tw, K * N * sizeof(ulonglong2)));
        HEC_HIP(hipMalloc(&c.itw, K * N * sizeof(ulonglong2)));
        HEC_HIP(hipMemcpy(c.tw, tw.data(), K * N * sizeof(ulonglong2), hipMemcpyHostToDevice));
        HEC_HIP(hipMemcpy(c.itw, itw.data(), K * N * sizeof(ulonglong2), hipMemcpyHostToDevice));
        {   // split-input Shoup words a = w 2^31 mod q of tw / itw (integer primes; hec_device.h shoup_split_lazy)
            std::vector<u64> ta(K * N, 0), ita(K * N, 0);
            for (uint64_t i = 0; i < K; ++i) {
                if (c.hprimes[i].fp) continue;
                const u64 q = c.q[i];
                for (uint64_t k = 0; k < N; ++k) {
                    ta[i * N + k] = (u64)(((u128)tw[i * N + k].x << 31) % q);
                    ita[i * N + k] = (u64)(((u128)itw[i * N + k].x << 31) % q);
                }
            }
            HEC_HIP(hipMalloc(&c.tws, K * N * sizeof(u64)));
            HEC_HIP(hipMalloc(&c.itws, K * N * sizeof(u64)));
            HEC_HIP(hipMemcpy(c.tws, ta.data(), K * N * sizeof(u64), hipMemcpyHostToDevice));
            HEC_HIP(hipMemcpy(c.itws, ita.data(), K * N * sizeof(u64), hipMemcpyHostToDevice));
        }
        const u64 P = c.q[K - 1];
        for (uint64_t i = 0; i < c.L; ++i) {
            const u64 q = c.q[i], pi = invm(P % q, q);
            c.p_inv.push_back(pi);
            c.p_inv_q.push_back(shoupq(pi, q));
            c.p_half_mod.push_back((P >> 1) % q);
        }
        c.ql_inv.assign(c.L + 1, {});
        c.ql_inv_q.assign(c.L + 1, {});
        c.ql_half_mod.assign(c.L + 1, {});
        for (uint64_t l = 2; l <= c.L; ++l)
            for (uint64_t i = 0; i + 1 < l; ++i) {
                const u64 q = c.q[i], ql = c.q[l - 1], v = invm(ql % q, q);
                c.ql_inv[l].push_back(v);
                c.ql_inv_q[l].push_back(shoupq(v, q));
                c.ql_half_mod[l].push_back((ql >> 1) % q);
            }
        // the tables went up with blocking copies on the null stream, which the non-blocking context stream does
        // not wait for: finish them before any kernel can read them
        HEC_HIP(hipDeviceSynchronize());
        ctx->gen = ctx_register(ctx);
        *out = ctx;
    });
}

int hec_context_destroy(hec_context *ctx)
{
    return guard([&] {
        if (!ctx) return;
        ctx_unregister(ctx);
        Ctx &c = ctx->c;
        (void)hipSetDevice(c.device);
        (void)hipStreamSynchronize(c.stream);
        for (hec_context *l : ctx->lanes) free_lane(l);
        if (ctx->lanes_start) (void)hipEventDestroy(ctx->lanes_start);
        delete ctx->comm;
        c.ws.release();
        (void)hipFree(c.primes);
        (void)hipFree(c.imap);
        (void)hipFree(c.psipow);
        (void)hipFree(c.cji);
        (void)hipFree(c.zflag);
        (void)hipFree(c.tw);
        (void)hipFree(c.itw);
        (void)hipFree(c.twb);
        (void)hipFree(c.itwb);
        (void)hipFree(c.tws);
        (void)hipFree(c.itws);
        (void)hipFree(c.twbs);
        for (double *p : {c.twf, c.itwf, c.twbf, c.itwbf}) (void)hipFree(p);
        (void)hipFree(c.enc_map);
        (void)hipFree(c.enc_tw);
        if (c.own_stream) (void)hipStreamDestroy(c.stream);
        for (hipEvent_t e : c.ev_pool) (void)hipEventDestroy(e);
        delete ctx;
    });
}

int hec_context_set_stream(hec_context *ctx, void *stream)
{
    return guard([&] {
        set_device(ctx);
        Ctx &c = ctx->c;
        HEC_HIP(hipStreamSynchronize(c.stream));
        if (c.own_stream) HEC_HIP(hipStreamDestroy(c.stream));
        if (stream) {
            c.stream = (hipStream_t)stream;
            c.own_stream = false;
        } else {
            HEC_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
            c.own_stream = true;
        }
    });
}

int hec_context_set_option(hec_context *ctx, const char *name, int64_t value)
{
    return guard([&] {
        need(ctx && name, "null argument");
        set_device(ctx);
        const std::string n(name);
        // the enumerated knobs take only their listed values (a typo in an A/B value must not pass as
        // another schedule)
        auto in = [&](int64_t lo, int64_t hi) {
            if (value < lo || value > hi)
                throw std::invalid_argument("option " + n + " takes " + std::to_string(lo) + ".." + std::to_string(hi));
            return (int)value;
        };
        auto apply = [&](Ctx &c) {
            if (n == "lanes") c.lanes = (int)std::max<int64_t>(1, value);
            else if (n == "lane_min_batch") c.lane_min_batch = (int)std::max<int64_t>(1, value);
            else if (n == "poison") c.poison = value != 0;
            else if (n == "lane_serial") c.lane_serial = value != 0;
            else if (n == "debug_lanes") c.debug_lanes = value != 0;
            else if (n == "kernel_memops") c.kernel_memops = value != 0;
            else if (n == "split_bfly") c.split_bfly = in(0, 4);
            else if (n == "nttb_shfl") c.nttb_shfl = in(0, 2);
            else if (n == "nttb_shfl_dr") c.nttb_shfl_dr = in(0, 1);
            else if (n == "hmac_int") c.hmac_int = in(0, 1);
            else if (n == "moddown1") c.moddown1 = in(0, 1);
            else if (n == "nt_e") c.nt_e = in(0, 1);
            else if (n == "bmac_split") c.bmac_split = value != 0;
            else if (n == "hoist") c.hoist = value != 0;
            else if (n == "hoist_min") c.hoist_min_children = (int)std::max<int64_t>(1, value);
            else if (n == "hmac") c.hmac_cfg = in(0, 2);
            else if (n == "hmac_odd3") c.hmac_odd3 = in(0, 1);
            else if (n == "hoist_scan") c.hoist_scan = in(0, 1);
            else if (n == "fan") c.fan_out = value != 0;
            else if (n == "fuse_galois") c.fuse_galois = value != 0;
            else if (n == "fused_modup_mac") c.fused_modup_mac = value != 0;
            else if (n == "tensor_defer") c.tensor_defer_max = (int)std::max<int64_t>(1, value);
            else if (n == "tensor_bufs") c.tensor_defer_bufs = (int)std::max<int64_t>(1, value);
            else if (n == "tensor_xcd") c.tensor_xcd = (int)std::max<int64_t>(0, value);
            else throw std::invalid_argument("unknown option");
        };
        HEC_HIP(hipStreamSynchronize(ctx->c.stream));
        apply(ctx->c);
        for (hec_context *l : ctx->lanes) {  // the lanes hold copies of the knobs (make_lane)
            HEC_HIP(hipStreamSynchronize(l->c.stream));
            apply(l->c);
        }
    });
}

int hec_context_synchronize(hec_context *ctx)
{
    return guard([&] {
        set_device(ctx);
        HEC_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}
uint64_t hec_context_poly_degree(const hec_context *ctx) { return ctx ? ctx->c.N : 0; }
uint64_t hec_context_key_moduli(const hec_context *ctx) { return ctx ? ctx->c.K : 0; }

uint32_t hec_galois_elt_from_step(const hec_context *ctx, int step)
{
    u32 e = 0;
    if (guard([&] { e = elt_from_step(ctx->c, step); })) return 0;
    return e;
}

uint64_t hec_default_galois_elts(const hec_context *ctx, uint32_t *out)
{
    const u32 m = (u32)(2 * ctx->c.N);
    std::vector<u32> v{m - 1};
    u64 pos = 3, neg = invm(3, m);
    for (int i = 0; i < ctx->c.logN - 1; ++i) {  // SEAL GaloisTool::get_elts_all
        v.push_back((u32)pos);
        pos = (pos * pos) & (m - 1);
        v.push_back((u32)neg);
        neg = (neg * neg) & (m - 1);
    }
    if (out) std::memcpy(out, v.data(), v.size() * sizeof(u32));
    return v.size();
}

// ------------------------------------------------------------------ ciphertext / plaintext
int hec_ciphertext_create(hec_context *ctx, hec_ciphertext **out)
{
    return guard([&] {
        need(ctx && out, "null argument");
        auto *ct = new hec_ciphertext();
        ct->ctx = ctx;
        ct->ctx_gen = ctx->gen;
        *out = ct;
    });
}
int hec_ciphertext_destroy(hec_ciphertext *ct)
{
    return guard([&] {
        if (!ct) return;
        if (ct->d) {
            if (ctx_alive(ct->ctx, ct->ctx_gen)) {
                (void)hipSetDevice(ct->ctx->c.device);
                (void)hipStreamSynchronize(ct->ctx->c.stream);
            }
            (void)hipFree(ct->d);
        }
        delete ct;
    });
}
int hec_ciphertext_upload(hec_ciphertext *ct, const uint64_t *host, uint64_t size, uint64_t level, double scale)
{
    return guard([&] {
        need(ct && host, "null argument");
        Ctx &c = ct->ctx->c;
        set_device(ct->ctx);
        need(size >= 1 && level >= 1 && level <= c.K, "encrypted is not valid for encryption parameters");
        const std::size_t w = size * level * c.N;
        ensure(ct, w);
        HEC_HIP(hipMemcpyAsync(ct->d, host, w * sizeof(u64), hipMemcpyHostToDevice, c.stream));
        HEC_HIP(hipStreamSynchronize(c.stream));
        ct->size = size; ct->level = level; ct->scale = scale;
    });
}
int hec_ciphertext_download(const hec_ciphertext *ct, uint64_t *host)
{
    return guard([&] {
        need(ct && host && ct->d, "null argument");
        Ctx &c = ct->ctx->c;
        set_device(ct->ctx);
        const std::size_t w = ct->size * ct->level * c.N;
        HEC_HIP(hipMemcpyAsync(host, ct->d, w * sizeof(u64), hipMemcpyDeviceToHost, c.stream));
        HEC_HIP(hipStreamSynchronize(c.stream));
    });
}
int hec_ciphertext_info(const hec_ciphertext *ct, uint64_t *size, uint64_t *level, double *scale)
{
    return guard([&] {
        need(ct != nullptr, "null argument");
        if (size) *size = ct->size;
        if (level) *level = ct->level;
        if (scale) *scale = ct->scale;
    });
}
int hec_ciphertext_copy(hec_ciphertext *dst, const hec_ciphertext *src)
{
    return guard([&] {
        need(dst && src && dst->ctx == src->ctx, "null argument");
        set_device(dst->ctx);
        if (dst == src) return;
        const std::size_t w = src->size * src->level * src->ctx->c.N;
        ensure(dst, w);
        d2d(src->ctx->c, dst->d, src->d, w);
        dst->size = src->size; dst->level = src->level; dst->scale = src->scale;
    });
}
int hec_ciphertext_export_device(const hec_ciphertext *ct, void *dev_dst)
{
    return guard([&] {
        need(ct && dev_dst && ct->d, "null argument");
        set_device(ct->ctx);
        d2d(ct->ctx->c, dev_dst, ct->d, ct->size * ct->level * ct->ctx->c.N);
    });
}
int hec_ciphertext_import_device(hec_ciphertext *ct, const void *dev_src, uint64_t size, uint64_t level, double scale)
{
    return guard([&] {
        need(ct && dev_src, "null argument");
        set_device(ct->ctx);
        const std::size_t w = size * level * ct->ctx->c.N;
        ensure(ct, w);
        d2d(ct->ctx->c, ct->d, dev_src, w);
        ct->size = size; ct->level = level; ct->scale = scale;
    });
}
int hec_ciphertext_reduce(hec_context *ctx, hec_ciphertext *ct)
{
    return guard([&] {
        check_ct(ctx, ct);
        set_device(ctx);
        ew_reduce(ctx->c, ct->d, (int)ct->size, (int)ct->level);
    });
}
int hec_ciphertext_fill_uniform(hec_ciphertext *ct, uint64_t size, uint64_t level, double scale, uint64_t seed)
{
    return guard([&] {
        need(ct != nullptr, "null argument");
        Ctx &c = ct->ctx->c;
        set_device(ct->ctx);
        need(size >= 1 && level >= 1 && level <= c.L, "encrypted is not valid for encryption parameters");
        ensure(ct, size * level * c.N);
        fill_uniform(c, ct->d, (int)size, (int)level, 0, 0, seed);
        ct->size = size; ct->level = level; ct->scale = scale;
    });
}

int hec_plaintext_create(hec_context *ctx, hec_plaintext **out)
{
    return guard([&] {
        need(ctx && out, "null argument");
        auto *p = new hec_plaintext();
        p->ctx = ctx;
        p->ctx_gen = ctx->gen;
        *out = p;
    });
}
int hec_plaintext_destroy(hec_plaintext *pt)
{
    return guard([&] {
        if (!pt) return;
        if (pt->d) {
            if (ctx_alive(pt->ctx, pt->ctx_gen)) (void)hipStreamSynchronize(pt->ctx->c.stream);
            (void)hipFree(pt->d);
        }
        delete pt;
    });
}
int hec_plaintext_fill_uniform(hec_plaintext *pt, uint64_t level, double scale, uint64_t seed)
{
    return guard([&] {
        need(pt != nullptr, "null argument");
        Ctx &c = pt->ctx->c;
        set_device(pt->ctx);
        need(level >= 1 && level <= c.L, "plain is not valid for encryption parameters");
        const std::size_t w = level * c.N;
        if (pt->cap < w) {
            if (pt->d) HEC_HIP(hipFree(pt->d));
            pt->d = dalloc(w);
            pt->cap = w;
        }
        fill_uniform(c, pt->d, 1, (int)level, 0, 0, seed);
        pt->level = level; pt->scale = scale;
    });
}

int hec_plaintext_upload(hec_plaintext *pt, const uint64_t *host, uint64_t level, double scale)
{
    return guard([&] {
        need(pt && host, "null argument");
        Ctx &c = pt->ctx->c;
        set_device(pt->ctx);
        need(level >= 1 && level <= c.L, "plain is not valid for encryption parameters");
        const std::size_t w = level * c.N;
        if (pt->cap < w) {
            if (pt->d) HEC_HIP(hipFree(pt->d));
            pt->d = dalloc(w);
            pt->cap = w;
        }
        HEC_HIP(hipMemcpyAsync(pt->d, host, w * sizeof(u64), hipMemcpyHostToDevice, c.stream));
        HEC_HIP(hipStreamSynchronize(c.stream));
        pt->level = level; pt->scale = scale;
    });
}

int hec_plaintext_download(const hec_plaintext *pt, uint64_t *host)
{
    return guard([&] {
        need(pt && host, "null argument");
        need(pt->d != nullptr, "plain is not valid for encryption parameters");
        Ctx &c = pt->ctx->c;
        set_device(pt->ctx);
        HEC_HIP(hipMemcpyAsync(host, pt->d, pt->level * c.N * sizeof(u64), hipMemcpyDeviceToHost, c.stream));
        HEC_HIP(hipStreamSynchronize(c.stream));
    });
}

int hec_plaintext_info(const hec_plaintext *pt, uint64_t *level, double *scale)
{
    return guard([&] {
        need(pt != nullptr, "null argument");
        if (level) *level = pt->level;
        if (scale) *scale = pt->scale;
    });
}

// ------------------------------------------------------------------ CKKS encoder ----------
namespace {
// host tables of the GPU encoder (hec_encode.hip), built once per context, as SEAL 4.1's CKKSEncoder constructor
// builds them: matrix_reps_index_map_ (generator 3, bit-reversed positions) and inv_root_powers_[i] =
// conj(ComplexRoots(2N).get_root(bitrev(i - 1, logN) + 1)), where ComplexRoots holds (cos t, sin t),
// t = (i 6.283185307179586) / 2N for i <= 2N / 8 (glibc cos and sin as separate calls) and get_root extends them by
// the 8-fold symmetry
struct SealRoots {  // a class member: no C language linkage inside the C-ABI block
static std::complex<double> get(u64 m, const std::vector<std::complex<double>> &roots, u64 index)
{
    index &= m - 1;
    if (index <= m / 8) return roots[index];
    if (index <= m / 4) {
        const auto a = roots[m / 4 - index];
        return {a.imag(), a.real()};
    }
    if (index <= m / 2) {
        const auto a = get(m, roots, m / 2 - index);
        return {-a.real(), a.imag()};
    }
    if (index <= 3 * m / 4) {
        const auto a = get(m, roots, index - m / 2);
        return {-a.real(), -a.imag()};
    }
    const auto a = get(m, roots, m - index);
    return {a.real(), -a.imag()};
}
};
void encoder_tables(Ctx &c)
{
    if (c.enc_map) return;
    const u64 N = c.N, slots = N / 2, m = 2 * N;
    std::vector<u32> map(N);
    u64 pos = 1;
    for (u64 i = 0; i < slots; ++i) {
        map[i] = brev((u32)((pos - 1) >> 1), c.logN);
        map[slots + i] = brev((u32)((m - pos - 1) >> 1), c.logN);
        pos = (pos * 3) & (m - 1);
    }
    double (*volatile vcos)(double) = std::cos;  // never fused into sincos
    double (*volatile vsin)(double) = std::sin;
    std::vector<std::complex<double>> roots(m / 8 + 1);
    for (u64 i = 0; i <= m / 8; ++i) {
        const double t = ((double)i * 6.283185307179586) / (double)m;
        roots[i] = {vcos(t), vsin(t)};
    }
    std::vector<double> inv(2 * N, 0.0);
    for (u64 i = 1; i < N; ++i) {
        const auto r = SealRoots::get(m, roots, (u64)brev((u32)(i - 1), c.logN) + 1);
        inv[2 * i] = r.real();
        inv[2 * i + 1] = -r.imag();
    }
    u32 *dm = nullptr;
    double *dt = nullptr;
    HEC_HIP(hipMalloc(&dm, N * sizeof(u32)));
    HEC_HIP(hipMalloc(&dt, inv.size() * sizeof(double)));
    HEC_HIP(hipMemcpyAsync(dm, map.data(), N * sizeof(u32), hipMemcpyHostToDevice, c.stream));
    HEC_HIP(hipMemcpyAsync(dt, inv.data(), inv.size() * sizeof(double), hipMemcpyHostToDevice, c.stream));
    HEC_HIP(hipStreamSynchronize(c.stream));  // the host tables go out of scope
    c.enc_map = dm;
    c.enc_tw = dt;
}
}  // namespace

int hec_encode(hec_context *ctx, const double *re, const double *im, uint64_t n_values, uint64_t count, double scale,
               uint64_t level, hec_plaintext *const *out)
{
    return guard([&] {
        need(ctx && out && (re || n_values == 0), "null argument");
        Ctx &c = ctx->c;
        set_device(ctx);
        // argument checks in SEAL CKKSEncoder::encode_internal's order
        if (n_values > c.N / 2) throw std::invalid_argument("values has invalid size");
        if (level < 1 || level > c.L) throw std::invalid_argument("parms_id is not valid for encryption parameters");
        if (scale <= 0 || (int)std::log2(scale) >= c.total_bits(level)) throw std::invalid_argument("scale out of bounds");
        for (u64 v = 0; v < count; ++v) need(out[v] && out[v]->ctx == ctx, "plain is not valid for encryption parameters");
        if (count == 0) return;
        encoder_tables(c);
        const u64 N = c.N, nv = n_values;
        // chunks of vectors: the work area (2N doubles + level N residues per vector) stays under ~2 GiB
        const u64 per = 2 * N + level * N + 2 * nv + 1;
        const u64 chunk = std::max<u64>(1, std::min<u64>(count, (u64(1) << 28) / per));
        std::vector<u64> mx(chunk);
        for (u64 v0 = 0; v0 < count; v0 += chunk) {
            const u64 cnt = std::min(chunk, count - v0);
            Scratch s(c, cnt * per + 5 * 64);
            double *dre = reinterpret_cast<double *>(s.take(std::max<u64>(cnt * nv, 1)));
            double *dim = im ? reinterpret_cast<double *>(s.take(std::max<u64>(cnt * nv, 1))) : nullptr;
            double *work = reinterpret_cast<double *>(s.take(cnt * 2 * N));
            u64 *res = s.take(cnt * level * N), *dmx = s.take(cnt);
            if (nv) {
                HEC_HIP(hipMemcpyAsync(dre, re + v0 * nv, cnt * nv * sizeof(double), hipMemcpyHostToDevice, c.stream));
                if (im)
                    HEC_HIP(hipMemcpyAsync(dim, im + v0 * nv, cnt * nv * sizeof(double), hipMemcpyHostToDevice,
                                           c.stream));
            }
            encode_batch(c, dre, dim, nv, (int)cnt, scale, (int)level, work, res, dmx);
            HEC_HIP(hipMemcpyAsync(mx.data(), dmx, cnt * sizeof(u64), hipMemcpyDeviceToHost, c.stream));
            HEC_HIP(hipStreamSynchronize(c.stream));
            for (u64 v = 0; v < cnt; ++v) {
                double maxabs;
                std::memcpy(&maxabs, &mx[v], sizeof(double));
                // ceil(log2(max(max |Re|, 1))) + 1 >= total coeff-modulus bits -> throw (SEAL encode_internal; the
                // maximum is over the unrounded real parts); a non-finite value is rejected the same way
                if (!std::isfinite(maxabs)) throw std::invalid_argument("encoded values are too large");
                const int max_bits = (int)std::ceil(std::log2(std::max(maxabs, 1.0))) + 1;
                if (max_bits >= c.total_bits(level)) throw std::invalid_argument("encoded values are too large");
            }
            for (u64 v = 0; v < cnt; ++v) {
                hec_plaintext *pt = out[v0 + v];
                const std::size_t w = level * N;
                if (pt->cap < w) {
                    if (pt->d) HEC_HIP(hipFree(pt->d));
                    pt->d = dalloc(w);
                    pt->cap = w;
                }
                d2d(c, pt->d, res + v * w, w);
                pt->level = level;
                pt->scale = scale;
            }
            HEC_HIP(hipStreamSynchronize(c.stream));  // the next chunk reuses the workspace
        }
    });
}

// the residue mod q of a non-negative integer-valued double a (exactly the integer a, as SEAL's 64-bit, 128-bit
// (fmod / division by 2^64) and multi-word decompositions give it)
static u64 exact_residue(double a, u64 q)
{
    if (a < 18446744073709551616.0) return (u64)a % q;
    int e = 0;
    const double f = std::frexp(a, &e);  // a = f 2^e, 0.5 <= f < 1, e > 64
    u64 r = (u64)std::ldexp(f, 53) % q, pw = 2 % q;
    for (int k = e - 53; k > 0; k >>= 1) {  // r *= 2^(e - 53) mod q
        if (k & 1) r = (u64)((unsigned __int128)r * pw % q);
        pw = (u64)((unsigned __int128)pw * pw % q);
    }
    return r;
}

int hec_encode_scalar(hec_context *ctx, double value, double scale, uint64_t level, hec_plaintext *out)
{
    return guard([&] {
        need(ctx && out, "null argument");
        Ctx &c = ctx->c;
        set_device(ctx);
        // SEAL 4.1 CKKSEncoder::encode_internal(double value, parms_id, scale, destination), in its order
        if (level < 1 || level > c.L) throw std::invalid_argument("parms_id is not valid for encryption parameters");
        need(out->ctx == ctx, "plain is not valid for encryption parameters");
        const int total = c.total_bits(level);
        if (scale <= 0 || (int)std::log2(scale) >= total) throw std::invalid_argument("scale out of bounds");
        value *= scale;
        // coeff_bit_count = int(log2 |value|) + 2; a zero value passes (SEAL's cast of -inf), a non-finite one is
        // rejected (SEAL would cast NaN / inf to int: undefined behaviour)
        if (!std::isfinite(value)) throw std::invalid_argument("encoded value is too large");
        if (value != 0.0 && (int)std::log2(std::fabs(value)) + 2 >= total)
            throw std::invalid_argument("encoded value is too large");
        const double cd = std::round(value);
        const bool neg = std::signbit(cd);
        const double a = std::fabs(cd);
        u64 words[HEC_MAXL + 1];
        for (std::size_t j = 0; j < level; ++j) {
            const u64 q = c.q[j], r = exact_residue(a, q);
            words[j] = neg && r ? q - r : r;  // negate_uint_mod
        }
        // the constant polynomial in NTT form: every coefficient of limb j is the residue (SEAL's fill_n)
        const std::size_t w = level * c.N;
        if (out->cap < w) {
            if (out->d) HEC_HIP(hipFree(out->d));
            out->d = dalloc(w);
            out->cap = w;
        }
        fill_limbs(c, out->d, (int)level, words);
        out->level = level;
        out->scale = scale;
    });
}

// ------------------------------------------------------------------ keys ------------------
static std::size_t key_words(const Ctx &c) { return c.L * 2 * c.K * c.N; }

int hec_kswitch_key_upload(hec_context *ctx, const uint64_t *host, hec_kswitch_key **out)
{
    return guard([&] {
        need(ctx && host && out, "null argument");
        set_device(ctx);
        auto *k = new hec_kswitch_key();
        k->ctx = ctx;
        k->ctx_gen = ctx->gen;
        k->d = dalloc(key_words(ctx->c));
        // on the context stream, drained before the host buffer may go (a pageable hipMemcpy on the null stream is
        // not ordered with the non-blocking context stream)
        HEC_HIP(hipMemcpyAsync(k->d, host, key_words(ctx->c) * sizeof(u64), hipMemcpyHostToDevice, ctx->c.stream));
        HEC_HIP(hipStreamSynchronize(ctx->c.stream));
        *out = k;
    });
}
int hec_kswitch_key_download(const hec_kswitch_key *key, uint64_t *host)
{
    return guard([&] {
        need(key && host, "null argument");
        set_device(key->ctx);
        Ctx &c = key->ctx->c;
        HEC_HIP(hipMemcpyAsync(host, key->d, key_words(c) * sizeof(u64), hipMemcpyDeviceToHost, c.stream));
        HEC_HIP(hipStreamSynchronize(c.stream));
    });
}
int hec_kswitch_key_fill_uniform(hec_context *ctx, uint64_t seed, hec_kswitch_key **out)
{
    return guard([&] {
        need(ctx && out, "null argument");
        set_device(ctx);
        Ctx &c = ctx->c;
        auto *k = new hec_kswitch_key();
        k->ctx = ctx;
        k->ctx_gen = ctx->gen;
        k->d = dalloc(key_words(c));
        fill_uniform(c, k->d, (int)(c.L * 2), (int)c.K, 0, 0, seed);
        HEC_HIP(hipStreamSynchronize(c.stream));
        *out = k;
    });
}
int hec_kswitch_key_destroy(hec_kswitch_key *key)
{
    return guard([&] {
        if (!key) return;
        if (ctx_alive(key->ctx, key->ctx_gen)) (void)hipStreamSynchronize(key->ctx->c.stream);
        (void)hipFree(key->d);
        delete key;
    });
}
int hec_galois_keys_create(hec_context *ctx, hec_galois_keys **out)
{
    return guard([&] {
        need(ctx && out, "null argument");
        auto *g = new hec_galois_keys();
        g->ctx = ctx;
        g->ctx_gen = ctx->gen;
        *out = g;
    });
}
static void gk_check_elt(const Ctx &c, u32 elt)
{
    need((elt & 1) && elt < 2 * c.N, "Galois element is not valid");
}
int hec_galois_keys_add(hec_galois_keys *gk, uint32_t elt, const uint64_t *host)
{
    return guard([&] {
        need(gk && host, "null argument");
        Ctx &c = gk->ctx->c;
        set_device(gk->ctx);
        gk_check_elt(c, elt);
        HEC_HIP(hipStreamSynchronize(c.stream));  // a replaced key may still be read by enqueued work
        u64 *&d = gk->keys[elt];
        if (!d) d = dalloc(key_words(c));
        gk->drop_kw(elt);
        HEC_HIP(hipMemcpyAsync(d, host, key_words(c) * sizeof(u64), hipMemcpyHostToDevice, c.stream));
        HEC_HIP(hipStreamSynchronize(c.stream));
    });
}
int hec_galois_keys_download(const hec_galois_keys *gk, uint32_t elt, uint64_t *host)
{
    return guard([&] {
        need(gk && host, "null argument");
        set_device(gk->ctx);
        Ctx &c = gk->ctx->c;
        const auto it = gk->keys.find(elt);
        need(it != gk->keys.end(), "Galois key not present");
        HEC_HIP(hipMemcpyAsync(host, it->second, key_words(c) * sizeof(u64), hipMemcpyDeviceToHost, c.stream));
        HEC_HIP(hipStreamSynchronize(c.stream));
    });
}
int hec_galois_keys_add_uniform(hec_galois_keys *gk, uint32_t elt, uint64_t seed)
{
    return guard([&] {
        need(gk != nullptr, "null argument");
        Ctx &c = gk->ctx->c;
        set_device(gk->ctx);
        gk_check_elt(c, elt);
        HEC_HIP(hipStreamSynchronize(c.stream));
        u64 *&d = gk->keys[elt];
        if (!d) d = dalloc(key_words(c));
        gk->drop_kw(elt);
        fill_uniform(c, d, (int)(c.L * 2), (int)c.K, 0, 0, seed);
        HEC_HIP(hipStreamSynchronize(c.stream));
    });
}
int hec_galois_keys_has(const hec_galois_keys *gk, uint32_t elt) { return gk && gk->keys.count(elt) ? 1 : 0; }
int hec_galois_keys_destroy(hec_galois_keys *gk)
{
    return guard([&] {
        if (!gk) return;
        debug_key_tables_forget(gk);
        if (ctx_alive(gk->ctx, gk->ctx_gen)) (void)hipStreamSynchronize(gk->ctx->c.stream);
        for (auto &kv : gk->keys) (void)hipFree(kv.second);
        for (auto &kv : gk->negw) (void)hipFree(kv.second);
        for (auto &kv : gk->kw) (void)hipFree(kv.second);
        for (auto &kv : gk->mkey) (void)hipFree(kv.second);
        delete gk;
    });
}

// ------------------------------------------------------------------ evaluator -------------
// ---------------------------------------------------------------- SEAL wire format on device objects
namespace {
void seal_rc(int rc)
{
    if (rc == HEC_EINVAL) throw std::invalid_argument(hec_seal_last_error());
    if (rc != HEC_OK) throw std::logic_error(hec_seal_last_error());
}
}  // namespace

int hec_ciphertext_load_seal(hec_ciphertext *ct, const void *bytes, uint64_t nbytes, uint64_t *consumed)
{
    return guard([&] {
        need(ct && bytes, "null argument");
        Ctx &c = ct->ctx->c;
        uint64_t size = 0, level = 0, N = 0, pid[4], used = 0;
        double scale = 0;
        // the context's data-level primes expand a seeded object (client.cpp:113-114 sends those)
        seal_rc(hec_seal_ciphertext_load_ex(bytes, nbytes, c.q.data(), c.L, &size, &level, &N, &scale, pid, nullptr, 0,
                                            &used));
        // Ciphertext::load(context, ...): the data must be valid for the context (is_valid_for)
        need(N == c.N && level >= 1 && level <= c.L && size >= 2, "ciphertext data is invalid");
        uint64_t want[4];
        seal_rc(hec_seal_parms_id(c.N, c.q.data(), level, want));
        need(std::memcmp(want, pid, 32) == 0, "ciphertext data is invalid");
        std::vector<u64> host(size * level * N);
        seal_rc(hec_seal_ciphertext_load_ex(bytes, nbytes, c.q.data(), c.L, nullptr, nullptr, nullptr, nullptr, nullptr,
                                            host.data(), host.size(), nullptr));
        const int rc = hec_ciphertext_upload(ct, host.data(), size, level, scale);
        if (rc != HEC_OK) throw std::logic_error(hec_last_error());
        if (consumed) *consumed = used;
    });
}

int hec_ciphertext_save_seal(const hec_ciphertext *ct, int compr_mode, void *out, uint64_t cap, uint64_t *written)
{
    return guard([&] {
        need(ct && ct->d, "null argument");
        const Ctx &c = ct->ctx->c;
        std::vector<u64> host(ct->size * ct->level * c.N);
        const int rc = hec_ciphertext_download(ct, host.data());
        if (rc != HEC_OK) throw std::logic_error(hec_last_error());
        seal_rc(hec_seal_ciphertext_save(host.data(), ct->size, ct->level, c.N, ct->scale, c.q.data(), compr_mode, out,
                                         cap, written));
    });
}

// Decompressed-size limit of a KSwitchKeys object loaded into this context (the bytes come from a client socket,
// server.cpp:110-122): `lists` key lists of L PublicKeys of u64[2][K][N], the object's N list-length words, and at
// most 256 B of SEALHeader / parms_id / ciphertext metadata per PublicKey.  The loader inflates the whole object into
// host memory before parsing it, so the default number of non-empty GaloisKeys lists is a fixed cap that does not
// depend on the device: four times SEAL's default set (create_galois_keys(), the reference's only form:
// matrix_operations.cpp:771,872,1064, holds 2 log2(N) - 1 lists), at least 64, at most N, and no more than half of the
// host's available physical memory can hold.  The same bound applies whether the object is compressed (the inflate
// budget) or not (counted as the lists are parsed).  hec_galois_keys_load_seal_ex takes an explicit limit instead.
static uint64_t galois_lists_default(const Ctx &c)
{
    const uint64_t logn = (uint64_t)__builtin_ctzll(c.N);
    uint64_t lists = std::min<uint64_t>(c.N, std::max<uint64_t>(64, 4 * (2 * logn - 1)));
    const long pages = sysconf(_SC_AVPHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
    if (pages > 0 && psz > 0) {
        const uint64_t per = c.L * (2 * c.K * c.N * 8 + 256);
        lists = std::min<uint64_t>(lists, std::max<uint64_t>(1, (uint64_t)pages * (uint64_t)psz / 2 / per));
    }
    return lists;
}
static uint64_t seal_keys_max_bytes(const Ctx &c, uint64_t lists)
{
    return lists * c.L * (2 * c.K * c.N * 8 + 256) + c.N * 8 + 4096;
}

int hec_kswitch_key_load_seal(hec_context *ctx, const void *bytes, uint64_t nbytes, hec_kswitch_key **out,
                              uint64_t *consumed)
{
    return guard([&] {
        need(ctx && bytes && out, "null argument");
        const Ctx &c = ctx->c;
        uint64_t words = 0, used = 0, lists = 0;
        const uint64_t cap = seal_keys_max_bytes(c, 1);
        seal_rc(hec_seal_kswitch_keys_load_ex(bytes, nbytes, 0, cap, &lists, nullptr, 0, &words, &used));
        need(lists >= 1 && words == c.L * 2 * c.K * c.N, "relin_keys is not valid for encryption parameters");
        std::vector<u64> host(words);
        seal_rc(hec_seal_kswitch_keys_load_ex(bytes, nbytes, 0, cap, nullptr, host.data(), words, nullptr, nullptr));
        const int rc = hec_kswitch_key_upload(ctx, host.data(), out);
        if (rc != HEC_OK) throw std::logic_error(hec_last_error());
        if (consumed) *consumed = used;
    });
}

int hec_galois_keys_load_seal_ex(hec_galois_keys *gk, const void *bytes, uint64_t nbytes, uint64_t max_lists,
                                 uint64_t *consumed)
{
    return guard([&] {
        need(gk && bytes, "null argument");
        need(gk->ctx, "null argument");
        set_device(gk->ctx);
        struct Visit {
            hec_galois_keys *gk;
            uint64_t max_lists, seen = 0;
            std::string err;
            int rc = HEC_OK;
        } v{gk, max_lists ? std::min<uint64_t>(max_lists, gk->ctx->c.N) : galois_lists_default(gk->ctx->c)};
        // one pass over the object: GaloisKeys::get_index(elt) = (elt - 1) / 2, every non-empty list uploaded as it
        // is parsed
        auto cb = [](void *user, uint64_t index, const uint64_t *words, uint64_t nwords) -> int {
            auto *st = static_cast<Visit *>(user);
            const Ctx &c = st->gk->ctx->c;
            if (nwords != c.L * 2 * c.K * c.N) {
                st->err = "galois_keys is not valid for encryption parameters";
                return st->rc = HEC_EINVAL;
            }
            if (++st->seen > st->max_lists) {  // the uncompressed object's form of the inflate budget below
                st->err = "decompressed SEAL object exceeds the size limit";
                return st->rc = HEC_EINVAL;
            }
            const int rc = hec_galois_keys_add(st->gk, (uint32_t)(2 * index + 1), words);
            if (rc != HEC_OK) st->err = hec_last_error();
            return st->rc = rc;
        };
        uint64_t used = 0;
        const int rc = hec_seal_kswitch_keys_foreach_ex(bytes, nbytes, seal_keys_max_bytes(gk->ctx->c, v.max_lists),
                                                        cb, &v, nullptr, &used);
        if (v.rc != HEC_OK) {
            if (v.rc == HEC_EINVAL) throw std::invalid_argument(v.err);
            throw std::logic_error(v.err);
        }
        seal_rc(rc);
        if (consumed) *consumed = used;
    });
}

int hec_galois_keys_load_seal(hec_galois_keys *gk, const void *bytes, uint64_t nbytes, uint64_t *consumed)
{
    return hec_galois_keys_load_seal_ex(gk, bytes, nbytes, 0, consumed);
}

uint64_t hec_galois_keys_load_seal_default_lists(const hec_context *ctx)
{
    return ctx ? galois_lists_default(ctx->c) : 0;
}

int hec_negate_inplace(hec_context *ctx, hec_ciphertext *a)
{
    return guard([&] {
        check_ct(ctx, a);
        set_device(ctx);
        ew_negate(ctx->c, PolyArr{a->d, 0, a->level * ctx->c.N}, 1, (int)a->size, (int)a->level);
    });
}

static void add_sub(hec_context *ctx, hec_ciphertext *a, const hec_ciphertext *b, bool sub)
{
    check_ct(ctx, a);
    check_ct(ctx, b);
    set_device(ctx);
    need(a->level == b->level, "encrypted1 and encrypted2 parameter mismatch");
    need(are_close(a->scale, b->scale), "scale mismatch");
    Ctx &c = ctx->c;
    const u64 ps = a->level * c.N;
    const std::size_t mn = std::min(a->size, b->size), mx = std::max(a->size, b->size);
    if (mx > a->size) {  // grow a, keeping its polys
        if (a->cap < mx * ps) {
            u64 *nd = dalloc(mx * ps);
            d2d(c, nd, a->d, a->size * ps);
            HEC_HIP(hipStreamSynchronize(c.stream));
            HEC_HIP(hipFree(a->d));
            a->d = nd;
            a->cap = mx * ps;
        }
    }
    ew_add(c, PolyArr{a->d, 0, ps}, PolyArr{b->d, 0, ps}, PolyArr{a->d, 0, ps}, 1, (int)mn, (int)a->level,
           sub ? 1 : 0);
    if (b->size > a->size) {  // SEAL: copy (add) or negate (sub) the extra polys of b
        const int extra = (int)(b->size - a->size);
        if (sub)
            ew_add(c, PolyArr{a->d + a->size * ps, 0, ps}, PolyArr{b->d + a->size * ps, 0, ps},
                   PolyArr{a->d + a->size * ps, 0, ps}, 1, extra, (int)a->level, 2);
        else
            d2d(c, a->d + a->size * ps, b->d + a->size * ps, extra * ps);
    }
    a->size = mx;
}
int hec_add_inplace(hec_context *ctx, hec_ciphertext *a, const hec_ciphertext *b)
{
    return guard([&] { add_sub(ctx, a, b, false); });
}
int hec_sub_inplace(hec_context *ctx, hec_ciphertext *a, const hec_ciphertext *b)
{
    return guard([&] { add_sub(ctx, a, b, true); });
}

static void plain_addsub(hec_context *ctx, hec_ciphertext *a, const hec_plaintext *p, bool sub)
{
    check_ct(ctx, a);
    need(p && p->ctx == ctx && p->d, "plain is not valid for encryption parameters");
    set_device(ctx);
    need(a->level == p->level, "encrypted and plain parameter mismatch");
    need(are_close(a->scale, p->scale), "scale mismatch");
    const u64 ps = a->level * ctx->c.N;
    ew_add(ctx->c, PolyArr{a->d, 0, ps}, PolyArr{p->d, 0, ps}, PolyArr{a->d, 0, ps}, 1, 1, (int)a->level,
           sub ? 1 : 0);
}
int hec_add_plain_inplace(hec_context *ctx, hec_ciphertext *a, const hec_plaintext *p)
{
    return guard([&] { plain_addsub(ctx, a, p, false); });
}
int hec_sub_plain_inplace(hec_context *ctx, hec_ciphertext *a, const hec_plaintext *p)
{
    return guard([&] { plain_addsub(ctx, a, p, true); });
}
int hec_multiply_plain_inplace(hec_context *ctx, hec_ciphertext *a, const hec_plaintext *p)
{
    return guard([&] {
        check_ct(ctx, a);
        need(p && p->ctx == ctx && p->d, "plain is not valid for encryption parameters");
        set_device(ctx);
        need(a->level == p->level, "encrypted_ntt and plain_ntt parameter mismatch");
        const double ns = a->scale * p->scale;
        need(scale_ok(ctx->c, ns, a->level), "scale out of bounds");
        ew_mul_plain(ctx->c, PolyArr{a->d, 0, 0}, p->d, (int)a->size, (int)a->level);
        a->scale = ns;
    });
}

static void multiply(hec_context *ctx, hec_ciphertext *a, const hec_ciphertext *b)
{
    check_ct(ctx, a);
    check_ct(ctx, b);
    set_device(ctx);
    need(a->level == b->level, "encrypted1 and encrypted2 parameter mismatch");
    const double ns = a->scale * b->scale;
    need(scale_ok(ctx->c, ns, a->level), "scale out of bounds");
    Ctx &c = ctx->c;
    const std::size_t ds = a->size + b->size - 1, ps = a->level * c.N;
    Scratch s(c, ds * ps + 64);
    u64 *tmp = s.take(ds * ps);
    ct_multiply(c, a->d, (int)a->size, b->d, (int)b->size, tmp, (int)a->level);
    if (a->cap < ds * ps) {
        HEC_HIP(hipStreamSynchronize(c.stream));
        HEC_HIP(hipFree(a->d));
        a->d = dalloc(ds * ps);
        a->cap = ds * ps;
    }
    d2d(c, a->d, tmp, ds * ps);
    a->size = ds;
    a->scale = ns;
}
int hec_multiply_inplace(hec_context *ctx, hec_ciphertext *a, const hec_ciphertext *b)
{
    return guard([&] { multiply(ctx, a, b); });
}
int hec_square_inplace(hec_context *ctx, hec_ciphertext *a)
{
    return guard([&] { multiply(ctx, a, a); });
}

int hec_relinearize_inplace(hec_context *ctx, hec_ciphertext *a, const hec_kswitch_key *rk)
{
    return guard([&] {
        check_ct(ctx, a);
        need(rk && rk->ctx == ctx, "relin_keys is not valid for encryption parameters");
        set_device(ctx);
        if (a->size == 2) return;
        need(a->size == 3, "not enough relinearization keys");
        Ctx &c = ctx->c;
        const u64 ps = a->level * c.N;
        Scratch s(c, ks_words(c, 1, a->level));
        const PolyArr io{a->d, 0, ps};
        keyswitch(c, s, PolyArr{a->d + 2 * ps, 0, 0}, rk->d, io, 2, io, 1, (int)a->level);
        a->size = 2;
    });
}

int hec_rescale_to_next_inplace(hec_context *ctx, hec_ciphertext *a)
{
    return guard([&] {
        check_ct(ctx, a);
        set_device(ctx);
        if (a->level == 1) throw std::invalid_argument("end of modulus switching chain reached");
        Ctx &c = ctx->c;
        const std::size_t l = a->level, N = c.N, nk = a->size, So = nk * (l - 1) * N;
        Scratch s(c, rescale_words(c, 1, nk, l) + So + 64);
        u64 *O = s.take(So);
        rescale_batch(c, s, PolyArr{a->d, nk * l * N, l * N}, 1, (int)nk, (int)l, PolyArr{O, So, (l - 1) * N});
        d2d(c, a->d, O, So);
        a->level = l - 1;
        a->scale = a->scale / (double)c.q[l - 1];
    });
}

int hec_mod_switch_to_next_inplace(hec_context *ctx, hec_ciphertext *a)
{
    return guard([&] {
        check_ct(ctx, a);
        set_device(ctx);
        if (a->level == 1) throw std::invalid_argument("end of modulus switching chain reached");
        need(scale_ok(ctx->c, a->scale, a->level - 1), "scale out of bounds");
        Ctx &c = ctx->c;
        const std::size_t l = a->level, N = c.N, nk = a->size;
        Scratch s(c, nk * (l - 1) * N + 64);
        u64 *O = s.take(nk * (l - 1) * N);
        for (std::size_t k = 0; k < nk; ++k) d2d(c, O + k * (l - 1) * N, a->d + k * l * N, (l - 1) * N);
        d2d(c, a->d, O, nk * (l - 1) * N);
        a->level = l - 1;
    });
}

static void galois_single(hec_context *ctx, hec_ciphertext *a, const std::vector<u32> &elts, const hec_galois_keys *gk)
{
    Ctx &c = ctx->c;
    const std::size_t l = a->level, N = c.N;
    Scratch s(c, ks_words(c, 1, l) + 2 * l * N + 128);
    const PolyArr x{a->d, 0, l * N};
    for (u32 e : elts) galois_ks(c, s, x, x, 1, (int)l, e, gk->keys.at(e));
}

int hec_rotate_vector_inplace(hec_context *ctx, hec_ciphertext *a, int steps, const hec_galois_keys *gk)
{
    return guard([&] {
        check_ct(ctx, a);
        need(gk && gk->ctx == ctx, "galois_keys is not valid for encryption parameters");
        set_device(ctx);
        if (steps == 0) return;  // Evaluator::rotate_internal
        need(a->size == 2, "encrypted size must be 2");
        std::vector<u32> elts;
        rotation_elts(ctx->c, steps, *gk, elts);
        galois_single(ctx, a, elts, gk);
    });
}

int hec_apply_galois_inplace(hec_context *ctx, hec_ciphertext *a, uint32_t elt, const hec_galois_keys *gk)
{
    return guard([&] {
        check_ct(ctx, a);
        need(gk && gk->ctx == ctx, "galois_keys is not valid for encryption parameters");
        set_device(ctx);
        need(gk->keys.count(elt) > 0, "Galois key not present");
        gk_check_elt(ctx->c, elt);
        need(a->size == 2, "encrypted size must be 2");
        galois_single(ctx, a, {elt}, gk);
    });
}

// ------------------------------------------------------------------ he::linalg ------------
int hec_matmul_diag_col(hec_context *ctx, const hec_ciphertext *const *diags, uint64_t n,
                        const hec_ciphertext *const *cols, uint64_t p, const hec_kswitch_key *rk,
                        const hec_galois_keys *gk, hec_ciphertext *const *out)
{
    return guard([&] {
        set_device(ctx);
        need(diags && cols && out, "null argument");
        std::vector<std::size_t> js(n);
        for (std::size_t j = 0; j < n; ++j) js[j] = j;
        matvec_lanes(ctx, diags, nullptr, n, js, cols, p, rk, gk, true, out);
    });
}

int hec_matmul_diag_col_partial(hec_context *ctx, const hec_ciphertext *const *diags, uint64_t n, uint64_t j_begin,
                                uint64_t j_end, const hec_ciphertext *const *cols, uint64_t p,
                                const hec_galois_keys *gk, hec_ciphertext *const *acc_out)
{
    return guard([&] {
        set_device(ctx);
        need(diags && cols && acc_out, "null argument");
        need(j_begin < j_end && j_end <= n, "empty matrix operand");
        std::vector<std::size_t> js;
        for (uint64_t j = j_begin; j < j_end; ++j) js.push_back(j);
        matvec_lanes(ctx, diags, nullptr, n, js, cols, p, nullptr, gk, false, acc_out);
    });
}

int hec_matmul_diag_col_partial_set(hec_context *ctx, const hec_ciphertext *const *diags, uint64_t n,
                                    const uint64_t *j_idx, uint64_t nj, const hec_ciphertext *const *cols, uint64_t p,
                                    const hec_galois_keys *gk, hec_ciphertext *const *acc_out)
{
    return guard([&] {
        set_device(ctx);
        need(diags && cols && acc_out && j_idx, "null argument");
        std::vector<std::size_t> js(j_idx, j_idx + nj);
        std::sort(js.begin(), js.end());
        need(std::adjacent_find(js.begin(), js.end()) == js.end(), "duplicate diagonal index");
        matvec_lanes(ctx, diags, nullptr, n, js, cols, p, nullptr, gk, false, acc_out);
    });
}

int hec_matmul_diagpt_col(hec_context *ctx, const hec_plaintext *const *diags, uint64_t n,
                          const hec_ciphertext *const *cols, uint64_t p, const hec_galois_keys *gk,
                          hec_ciphertext *const *out)
{
    return guard([&] {
        set_device(ctx);
        need(diags && cols && out, "null argument");
        std::vector<std::size_t> js(n);
        for (std::size_t j = 0; j < n; ++j) js[j] = j;
        matvec_lanes(ctx, nullptr, diags, n, js, cols, p, nullptr, gk, true, out);
    });
}

int hec_matmul_finish(hec_context *ctx, hec_ciphertext *const *acc, uint64_t p, const hec_kswitch_key *rk,
                      hec_ciphertext *const *out)
{
    return guard([&] {
        set_device(ctx);
        need(acc && out && p >= 1, "null argument");
        need(rk && rk->ctx == ctx, "relin_keys is not valid for encryption parameters");
        Ctx &c = ctx->c;
        const std::size_t l = acc[0]->level, N = c.N, S3 = 3 * l * N, So = 2 * (l - 1) * N;
        for (uint64_t i = 0; i < p; ++i) {
            check_ct(ctx, acc[i]);
            need(acc[i]->size == 3 && acc[i]->level == l, "encrypted1 and encrypted2 parameter mismatch");
        }
        if (l < 2) throw std::invalid_argument("end of modulus switching chain reached");
        Scratch s(c, p * (S3 + So) + ks_words(c, p, l) + rescale_words(c, p, 2, l) + 256);
        u64 *A3 = s.take(p * S3), *O = s.take(p * So);
        for (uint64_t i = 0; i < p; ++i) d2d(c, A3 + i * S3, acc[i]->d, S3);
        const PolyArr Aa{A3, S3, l * N};
        keyswitch(c, s, PolyArr{A3 + 2 * l * N, S3, 0}, rk->d, Aa, 2, Aa, (int)p, (int)l);
        rescale_batch(c, s, Aa, (int)p, 2, (int)l, PolyArr{O, So, (l - 1) * N});
        std::vector<double> sc(p);
        for (uint64_t i = 0; i < p; ++i) sc[i] = acc[i]->scale / (double)c.q[l - 1];
        for (uint64_t i = 0; i < p; ++i) {
            ensure(out[i], So);
            d2d(c, out[i]->d, O + i * So, So);
            out[i]->size = 2; out[i]->level = l - 1; out[i]->scale = sc[i];
        }
    });
}

// ------------------------------------------------------------------ multi-GPU

int hec_plan_diagonal_shards(uint64_t N, uint64_t n, int world, const uint32_t *key_elts, uint64_t nkeys,
                             int32_t *rank_of_diag)
{
    return guard([&] {
        need(rank_of_diag && (key_elts || nkeys == 0), "null argument");
        need(N >= 1024 && N <= 65536 && !(N & (N - 1)), "poly_modulus_degree must be a power of two in [2^10, 2^16]");
        std::set<u32> keys(key_elts, key_elts + nkeys);
        const auto plan = plan_shards(N, n, world, keys);
        for (std::size_t r = 0; r < plan.size(); ++r)
            for (std::size_t j : plan[r]) rank_of_diag[j] = (int32_t)r;
    });
}

int hec_comm_unique_id(void *unique_id)
{
    return guard([&] {
        need(unique_id != nullptr, "null argument");
        ncclUniqueId id;
        nccl_check(rccl().get_unique_id(&id), "ncclGetUniqueId");
        std::memcpy(unique_id, &id, sizeof(id));
    });
}

int hec_comm_init(hec_context *ctx, int rank, int world, const void *unique_id)
{
    return guard([&] {
        set_device(ctx);
        need(world >= 1 && rank >= 0 && rank < world, "invalid rank / world");
        // the exchange adds `world` canonical residues < 2^60 in u64 (hec_matmul_diag_col_sharded); shard.py's
        // int64 exchange has the same bound
        need(world <= 8, "world must be at most 8 (exact u64 partial-sum exchange)");
        need(ctx->comm == nullptr, "communicator already initialised");
        if (world > 1 || unique_id) {  // world 1 with an id: a one-rank communicator (exercises the RCCL path)
            need(unique_id != nullptr, "null argument");
            ncclUniqueId id;
            std::memcpy(&id, unique_id, sizeof(id));
            ncclComm_t comm = nullptr;
            nccl_check(rccl().init_rank(&comm, world, id, rank), "ncclCommInitRank");
            ctx->comm = new RcclComm(comm);
        }
        ctx->rank = rank;
        ctx->world = world;
    });
}

int hec_comm_init_ops(hec_context *ctx, int rank, int world, const hec_comm_ops *ops)
{
    return guard([&] {
        set_device(ctx);
        need(world >= 1 && rank >= 0 && rank < world, "invalid rank / world");
        need(world <= 8, "world must be at most 8 (exact u64 partial-sum exchange)");
        need(ctx->comm == nullptr, "communicator already initialised");
        need(ops && ops->allreduce_f64 && ops->allreduce_u64_sum, "null argument");
        ctx->comm = new OpsComm(*ops);
        ctx->rank = rank;
        ctx->world = world;
    });
}

int hec_shard_agree(const hec_comm_ops *ops, int rank, int status, const char *reason, const double *scales,
                    uint64_t p, char *msg, uint64_t msg_cap)
{
    int agreed = HEC_OK;
    const int rc = guard([&] {
        need(ops && ops->allreduce_f64 && ops->allreduce_u64_sum && (p == 0 || scales || status), "null argument");
        need(status == HEC_OK || status == HEC_EINVAL || status == HEC_ELOGIC, "status must be HEC_OK / EINVAL / ELOGIC");
        need(rank >= 0 && rank < 255, "invalid rank / world");
        OpsComm cm(*ops);
        std::string m = reason ? reason : "";
        agreed = shard_agree(cm, rank, status, m, scales, p, nullptr);
        if (msg && msg_cap) {
            const std::size_t k = std::min<std::size_t>(m.size(), msg_cap - 1);
            std::memcpy(msg, m.data(), k);
            msg[k] = 0;
        }
    });
    return rc != HEC_OK ? rc : agreed;
}

int hec_context_comm(const hec_context *ctx, int *rank, int *world)
{
    if (!ctx) return HEC_EINVAL;
    if (rank) *rank = ctx->rank;
    if (world) *world = ctx->world;
    return ctx->comm ? 1 : 0;
}

int hec_matmul_diag_col_sharded(hec_context *ctx, const hec_ciphertext *const *diags, uint64_t n,
                                const hec_ciphertext *const *cols, uint64_t p, const hec_kswitch_key *rk,
                                const hec_galois_keys *gk, hec_ciphertext *const *out)
{
    return guard([&] {
        set_device(ctx);
        need(ctx->world == 1 || ctx->comm, "hec_comm_init has not been called");
        Ctx &c = ctx->c;
        // The argument checks run on this rank's planned diagonals only (the others are never dereferenced), then
        // the ranks agree on them before any data-path collective, so a bad argument on one rank is an error on
        // every rank instead of a rank left waiting in the exchange.  The product scales of the ranks' diagonals
        // are compared across ranks too (SEAL's add_inplace "scale mismatch" over the whole sum).
        std::vector<std::size_t> mine;
        std::vector<double> ps;
        int status = HEC_OK;
        std::string msg;
        try {
            need(diags && cols && out && n >= 1 && p >= 1, "empty matrix operand");
            need(gk && gk->ctx == ctx, "galois_keys is not valid for encryption parameters");
            std::set<u32> keys;
            for (const auto &kv : gk->keys) keys.insert(kv.first);
            mine = plan_shards(c.N, n, ctx->world, keys)[ctx->rank];
            ps = matvec_check(ctx, diags, nullptr, n, mine, cols, p, rk, gk, true);
        } catch (const std::invalid_argument &e) {
            status = HEC_EINVAL; msg = e.what();
        } catch (const std::logic_error &e) {
            status = HEC_ELOGIC; msg = e.what();
        }
        if (ctx->comm) status = shard_agree(*ctx->comm, ctx->rank, status, msg, ps.data(), p, c.stream);
        if (status == HEC_EINVAL) throw std::invalid_argument(msg);
        if (status) throw std::logic_error(msg);
        const std::size_t l = cols[0]->level, S3 = 3 * l * c.N;
        // this rank's size-3 partials over its trie subtrees of diagonals
        std::vector<hec_ciphertext> acc(p);
        std::vector<hec_ciphertext *> accp(p);
        for (uint64_t i = 0; i < p; ++i) { acc[i].ctx = ctx; acc[i].ctx_gen = ctx->gen; accp[i] = &acc[i]; }
        struct Free {
            std::vector<hec_ciphertext> &a;
            ~Free() { for (auto &x : a) if (x.d) (void)hipFree(x.d); }
        } free_acc{acc};
        matvec_lanes(ctx, diags, nullptr, n, mine, cols, p, nullptr, gk, false, accp.data());
        if (ctx->comm) {
            // the one exchange: a plain u64 sum of the world's canonical residues (< world 2^60 < 2^64), then
            // reduce mod q; every rank then holds the full accumulators (he_linalg.cpp:977-997 summed)
            u64 *buf = nullptr;
            HEC_HIP(hipMallocAsync((void **)&buf, p * S3 * sizeof(u64), c.stream));
            for (uint64_t i = 0; i < p; ++i) d2d(c, buf + i * S3, acc[i].d, S3);
            ctx->comm->allreduce_u64_sum(buf, p * S3, c.stream);
            ew_reduce(c, buf, (int)(3 * p), (int)l);
            for (uint64_t i = 0; i < p; ++i) d2d(c, acc[i].d, buf + i * S3, S3);
            HEC_HIP(hipFreeAsync(buf, c.stream));
        }
        // lazy relinearize + rescale (he_linalg.cpp:999-1002) of every output on every rank: p key switches
        // against the ~n/world rotations each rank ran, and no second collective
        const int rc = hec_matmul_finish(ctx, accp.data(), p, rk, out);
        if (rc != HEC_OK) throw std::logic_error(hec_last_error());
    });
}

int hec_matmul_col_colT(hec_context *ctx, const hec_ciphertext *const *A, uint64_t n, const hec_ciphertext *const *B,
                        uint64_t p, const hec_kswitch_key *rk, const hec_galois_keys *gk,
                        hec_ciphertext *const *out)
{
    return guard([&] {
        set_device(ctx);
        need(A && B && out && n >= 1 && p >= 1, "null argument");
        need(rk && rk->ctx == ctx && gk && gk->ctx == ctx, "keys are not valid for encryption parameters");
        Ctx &c = ctx->c;
        const std::size_t l = A[0]->level, N = c.N, S2 = 2 * l * N, S3 = 3 * l * N, So = 2 * (l - 1) * N;
        for (uint64_t j = 0; j < n; ++j) {
            check_ct(ctx, A[j]);
            check_ct(ctx, B[j]);
            need(A[j]->size == 2 && B[j]->size == 2, "encrypted size must be 2");
            need(A[j]->level == l && B[j]->level == l, "encrypted1 and encrypted2 parameter mismatch");
        }
        double sc = 0;
        for (uint64_t j = 0; j < n; ++j) {
            const double s = B[j]->scale * A[j]->scale;
            need(scale_ok(c, s, l), "scale out of bounds");
            if (j == 0) sc = s;
            else need(are_close(sc, s), "scale mismatch");
        }
        if (l < 2) throw std::invalid_argument("end of modulus switching chain reached");
        RotTrie trie;  // rotations rot(B[j], i) for all j share the trie over i
        {
            std::vector<u32> seq;
            for (uint64_t i = 0; i < p; ++i) {
                seq.clear();
                rotation_elts(c, (int)i, *gk, seq);
                trie.insert(seq, i);
            }
        }
        const int D = trie.depth;
        Scratch s(c, n * S2 * (D + 2) + p * (S3 + So) + ks_words(c, std::max<uint64_t>(n, p), l) + 2 * n * l * N +
                         rescale_words(c, p, 2, l) + (D + 80) * 64);
        TrieBufs bufs(s, D, 1, n * S2);
        u64 *Aw = s.take(n * S2), *AC = s.take(p * S3), *O = s.take(p * So);
        for (uint64_t j = 0; j < n; ++j) {
            d2d(c, Aw + j * S2, A[j]->d, S2);
            d2d(c, bufs.b[0][0] + j * S2, B[j]->d, S2);
        }
        const PolyArr Ba{bufs.b[0][0], S2, l * N}, Aa{Aw, S2, l * N};
        auto visit = [&](std::size_t i, PolyArr src) {  // out[i] = sum_j rot(B[j], i) (x) A[j]
            tensor_sum(c, src, Aa, AC + i * S3, l * N, (int)n, (int)l);
        };
        auto no_flush = [](const u64 *) {};
        walk_trie(c, s, trie, 0, Ba, 0, (int)n, (int)l, *gk, bufs, S2, visit, no_flush);
        const PolyArr Ca{AC, S3, l * N};
        keyswitch(c, s, PolyArr{AC + 2 * l * N, S3, 0}, rk->d, Ca, 2, Ca, (int)p, (int)l);
        rescale_batch(c, s, Ca, (int)p, 2, (int)l, PolyArr{O, So, (l - 1) * N});
        for (uint64_t i = 0; i < p; ++i) {
            ensure(out[i], So);
            d2d(c, out[i]->d, O + i * So, So);
            out[i]->size = 2; out[i]->level = l - 1; out[i]->scale = sc / (double)c.q[l - 1];
        }
    });
}

int hec_matrix_matmul(hec_context *ctx, const hec_ciphertext *const *A, uint64_t ar, uint64_t ac, int atr,
                      const hec_ciphertext *const *B, uint64_t br, uint64_t bc, int btr, const hec_kswitch_key *rk,
                      hec_ciphertext *const *out)
{
    return guard([&] {
        set_device(ctx);
        need(A && B && out, "null argument");
        need(rk && rk->ctx == ctx, "relin_keys is not valid for encryption parameters");
        Ctx &c = ctx->c;
        // Matrix::get_dims / ij_to_idx (he_linalg.cpp:25-28, 376-379)
        const uint64_t r1 = atr ? ac : ar, c1 = atr ? ar : ac, r2 = btr ? bc : br, c2 = btr ? br : bc;
        need(c1 == r2, "dimension mismatch");
        auto at = [](const hec_ciphertext *const *M, uint64_t rows, int tr, uint64_t i, uint64_t j) {
            return M[(tr ? j : i) + rows * (tr ? i : j)];
        };
        const std::size_t l = A[0]->level, N = c.N, S3 = 3 * l * N, So = 2 * (l - 1) * N;
        for (uint64_t k = 0; k < ar * ac; ++k) {
            check_ct(ctx, A[k]);
            need(A[k]->size == 2 && A[k]->level == l, "encrypted1 and encrypted2 parameter mismatch");
        }
        for (uint64_t k = 0; k < br * bc; ++k) {
            check_ct(ctx, B[k]);
            need(B[k]->size == 2 && B[k]->level == l, "encrypted1 and encrypted2 parameter mismatch");
        }
        if (l < 2) throw std::invalid_argument("end of modulus switching chain reached");
        const uint64_t no = r1 * c2;
        std::vector<double> sc(no);
        for (uint64_t j = 0; j < c2; ++j)
            for (uint64_t i = 0; i < r1; ++i)
                for (uint64_t k = 0; k < c1; ++k) {
                    const double s = at(A, ar, atr, i, k)->scale * at(B, br, btr, k, j)->scale;
                    need(scale_ok(c, s, l), "scale out of bounds");
                    if (k == 0) sc[i + r1 * j] = s;
                    else need(are_close(sc[i + r1 * j], s), "scale mismatch");
                }
        Scratch s(c, no * (S3 + So) + S3 + ks_words(c, no, l) + rescale_words(c, no, 2, l) + 512);
        u64 *AC = s.take(no * S3), *T = s.take(S3), *O = s.take(no * So);
        const PolyArr one{nullptr, 0, l * N};
        for (uint64_t j = 0; j < c2; ++j)
            for (uint64_t i = 0; i < r1; ++i) {  // he_linalg.cpp:218-228
                u64 *dst = AC + (i + r1 * j) * S3;
                for (uint64_t k = 0; k < c1; ++k) {
                    const hec_ciphertext *x = at(A, ar, atr, i, k), *y = at(B, br, btr, k, j);
                    ct_multiply(c, x->d, 2, y->d, 2, k == 0 ? dst : T, (int)l);
                    if (k) ew_add(c, PolyArr{dst, 0, l * N}, PolyArr{T, 0, l * N}, PolyArr{dst, 0, l * N}, 1, 3,
                                  (int)l, 0);
                }
            }
        (void)one;
        const PolyArr Ca{AC, S3, l * N};
        keyswitch(c, s, PolyArr{AC + 2 * l * N, S3, 0}, rk->d, Ca, 2, Ca, (int)no, (int)l);
        rescale_batch(c, s, Ca, (int)no, 2, (int)l, PolyArr{O, So, (l - 1) * N});
        for (uint64_t o = 0; o < no; ++o) {
            ensure(out[o], So);
            d2d(c, out[o]->d, O + o * So, So);
            out[o]->size = 2; out[o]->level = l - 1; out[o]->scale = sc[o] / (double)c.q[l - 1];
        }
    });
}

// ------------------------------------------------------------------ primitives ------------
int hec_ntt_forward(hec_context *ctx, uint64_t *d, uint64_t limb0, uint64_t nl, uint64_t np)
{
    return guard([&] {
        set_device(ctx);
        need(d && nl >= 1 && limb0 + nl <= ctx->c.K && nl <= HEC_MAXL + 1, "invalid limb range");
        int pm[HEC_MAXL + 1];
        for (uint64_t i = 0; i < nl; ++i) pm[i] = (int)(limb0 + i);
        // one scope per pass: each reads and writes every limb once (SURVEY 8(d)'s 2 N 8 B per limb-NTT)
        {
            ProfScope k(ctx->c, "k:k_ntt/fwd_a", 2.0 * nl * np);
            ntt_strided(ctx->c, false, d, nl * ctx->c.N, d, nl * ctx->c.N, (int)nl, pm, (int)(nl * np), 1, 1);
        }
        ProfScope k(ctx->c, "k:k_ntt/fwd_b", 2.0 * nl * np);
        ntt_strided(ctx->c, false, d, nl * ctx->c.N, d, nl * ctx->c.N, (int)nl, pm, (int)(nl * np), 1, 2);
    });
}
int hec_ntt_inverse(hec_context *ctx, uint64_t *d, uint64_t limb0, uint64_t nl, uint64_t np)
{
    return guard([&] {
        set_device(ctx);
        need(d && nl >= 1 && limb0 + nl <= ctx->c.K && nl <= HEC_MAXL + 1, "invalid limb range");
        int pm[HEC_MAXL + 1];
        for (uint64_t i = 0; i < nl; ++i) pm[i] = (int)(limb0 + i);
        {
            ProfScope k(ctx->c, "k:k_ntt/inv_b", 2.0 * nl * np);
            ntt_strided(ctx->c, true, d, nl * ctx->c.N, d, nl * ctx->c.N, (int)nl, pm, (int)(nl * np), 1, 1);
        }
        ProfScope k(ctx->c, "k:k_ntt/inv_a", 2.0 * nl * np);
        ntt_strided(ctx->c, true, d, nl * ctx->c.N, d, nl * ctx->c.N, (int)nl, pm, (int)(nl * np), 1, 2);
    });
}
int hec_dyadic_multiply(hec_context *ctx, const uint64_t *a, const uint64_t *b, uint64_t *out, uint64_t limb0,
                        uint64_t nl, uint64_t np)
{
    return guard([&] {
        set_device(ctx);
        need(a && b && out && limb0 + nl <= ctx->c.K, "invalid limb range");
        ProfScope k(ctx->c, "k:k_dyadic", 3.0 * nl * np);
        ew_dyadic(ctx->c, a, b, out, (int)limb0, (int)nl, (int)np);
    });
}
int hec_device_alloc(hec_context *ctx, uint64_t bytes, void **out)
{
    return guard([&] {
        set_device(ctx);
        HEC_HIP(hipMalloc(out, bytes ? bytes : 8));
    });
}
int hec_device_free(hec_context *ctx, void *p)
{
    return guard([&] {
        set_device(ctx);
        HEC_HIP(hipStreamSynchronize(ctx->c.stream));
        HEC_HIP(hipFree(p));
    });
}
int hec_memcpy_h2d(hec_context *ctx, void *dst, const void *src, uint64_t bytes)
{
    return guard([&] {
        set_device(ctx);
        HEC_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->c.stream));
        HEC_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}
int hec_memcpy_d2h(hec_context *ctx, void *dst, const void *src, uint64_t bytes)
{
    return guard([&] {
        set_device(ctx);
        HEC_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->c.stream));
        HEC_HIP(hipStreamSynchronize(ctx->c.stream));
    });
}

int hec_time_ntt_forward(hec_context *ctx, uint64_t *d, uint64_t nl, uint64_t np, int reps, double *ms)
{
    return guard([&] {
        set_device(ctx);
        need(d && ms && reps >= 1 && nl <= ctx->c.K, "invalid argument");
        Ctx &c = ctx->c;
        int pm[HEC_MAXL + 1];
        for (uint64_t i = 0; i < nl; ++i) pm[i] = (int)i;
        hipEvent_t e0, e1;
        HEC_HIP(hipEventCreate(&e0));
        HEC_HIP(hipEventCreate(&e1));
        HEC_HIP(hipEventRecord(e0, c.stream));
        for (int r = 0; r < reps; ++r)
            ntt_strided(c, false, d, nl * c.N, d, nl * c.N, (int)nl, pm, (int)(nl * np));
        HEC_HIP(hipEventRecord(e1, c.stream));
        HEC_HIP(hipEventSynchronize(e1));
        float t = 0;
        HEC_HIP(hipEventElapsedTime(&t, e0, e1));
        *ms = t / reps;
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    });
}

int hec_profile_enable(hec_context *ctx, int mode)
{
    return guard([&] {
        need(ctx != nullptr && mode >= 0 && mode <= 2, "invalid argument");
        Ctx &c = ctx->c;
        set_device(ctx);
        prof_resolve(c);
        c.prof_mode = mode;
        if (mode) c.prof_tab.clear();
    });
}
int hec_profile_read_ex(hec_context *ctx, const char *cls, double *total_ms, uint64_t *scopes, double *alg_bytes,
                        uint64_t *kernel_launches)
{
    return guard([&] {
        need(ctx && cls, "null");
        set_device(ctx);
        prof_resolve(ctx->c);
        auto it = ctx->c.prof_tab.find(cls);
        const bool has = it != ctx->c.prof_tab.end();
        if (total_ms) *total_ms = has ? it->second.ms : 0;
        if (scopes) *scopes = has ? it->second.n : 0;
        if (alg_bytes) *alg_bytes = has ? it->second.bytes : 0;
        if (kernel_launches) *kernel_launches = has ? it->second.kl : 0;
    });
}
uint64_t hec_profile_classes(hec_context *ctx, char *buf, uint64_t cap)
{
    if (!ctx) return 0;
    std::string all;
    try {
        set_device(ctx);
        prof_resolve(ctx->c);
    } catch (...) {
        return 0;
    }
    for (const auto &kv : ctx->c.prof_tab) all += kv.first + "\n";
    if (buf && cap) {
        const std::size_t n = std::min<std::size_t>(all.size(), cap - 1);
        std::memcpy(buf, all.data(), n);
        buf[n] = 0;
    }
    return all.size() + 1;
}
int hec_profile_read(hec_context *ctx, const char *cls, double *total_ms, uint64_t *launches)
{
    return guard([&] {
        need(ctx && cls, "null");
        set_device(ctx);
        prof_resolve(ctx->c);
        auto it = ctx->c.prof_tab.find(cls);
        if (total_ms) *total_ms = it == ctx->c.prof_tab.end() ? 0 : it->second.ms;
        if (launches) *launches = it == ctx->c.prof_tab.end() ? 0 : it->second.n;
    });
}

}  // extern "C"
