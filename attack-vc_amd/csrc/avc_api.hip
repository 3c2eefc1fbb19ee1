// libavc host side: C ABI (include/avc.h), weight packing, per-(B,T) workspace
// and launch plans, the on-device attack loop (hipGraph replay per iteration),
// and per-kernel HIP-event profiling for bench.py's roofline.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <string>
#include <vector>

#include "../../include/avc.h"
#include "avc_kernels.h"
#include "avc_ktime.h"

namespace avc {
template <int PREC, int WM, int WN, int WGM, int WGN, int KC, int MODE, int STRIDE>
__global__ void conv_gemm(const Problem* __restrict__ probs, int ksplit);
__global__ void splitk_reduce(const Problem* __restrict__ probs, int ksplit);
__global__ void se_head(HeadArgs A);
template <bool BW>
__global__ void se_head_v(HeadArgs A);
__global__ void attack_init(const float* vc, const float* ptb0, float* ptb, float* m, float* v, float* adv,
                            float eps, size_t n, int pgd);
template <int PREC, int SH>
__global__ void se_fwd_fused(FusedArgs A);
template <int PREC, int SH>
__global__ void se_bwd_fused(FusedArgs A);
template <int PREC, int SH>
__global__ void se_attack_fused(AtkArgs A);
__global__ void fz_step_add(int32_t* step, int n);
template <int PREC>
__global__ void lz_se_fwd(FusedArgs A, LongArgs L);
template <int PREC>
__global__ void lz_se_bwd(FusedArgs A, LongArgs L);
template <int PREC>
__global__ void lz_dec_fwd(DecArgs A, LongArgs L);
template <int PREC>
__global__ void lz_dec_bwd(DecArgs A, LongArgs L);
template <int PREC, int SH>
__global__ void dec_fwd_fused(DecArgs A);
template <int PREC, int SH>
__global__ void dec_bwd_fused(DecArgs A);
__global__ void dense_batched(DenseArgs D);
template <int NJ>
__global__ void dense_mfma(DenseArgs D);
__global__ void dense_lds(DenseArgs D);
__global__ void sn_power(SnArgs A);
__global__ void sn_scale(SnArgs A);
__global__ void hdr_compose(HdrArgs A);
__global__ void hdr_update(HdrArgs A);
__global__ void pm_conv(PmConvArgs P);
__global__ void pm_reduce(PmConvArgs P);
template <int CO>
__global__ void pm_cin1(PmConvArgs P);
template <int CI>
__global__ void pm_cout1(PmConvArgs P);
template <int CI>
__global__ void pm_cout1h(PmConvArgs P);
template <int MT, int MODE, int NT>
__global__ void pm_mfma(PmConvArgs P);
__global__ void vsm_gather(VsmArgs A);
__global__ void vsm_combine(VsmArgs A);
}  // namespace avc
#include "avc_fused_lds.h"

using namespace avc;

static thread_local std::string g_err;

static int fail(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return 1;
}

#define HIPCHK(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) return fail("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                                          __FILE__, __LINE__);                              \
    } while (0)

static inline int rup(int x, int m) { return (x + m - 1) / m * m; }
static inline int cdiv(int x, int m) { return (x + m - 1) / m; }

namespace {

struct DevBuf {
    float* p = nullptr;
    size_t n = 0;
};

// A conv layer of the SpeakerEncoder as stored by torch: W[co][ci][k], b[co].
struct HostConv {
    int co, ci, k;
    const float* W;
    const float* b;
};

enum LaunchKind {
    L_GEMM, L_HEAD, L_HEAD_V, L_FZ_FWD, L_FZ_BWD, L_DZ_FWD, L_DZ_BWD, L_DENSE, L_LZ_FWD, L_LZ_BWD, L_LZD_FWD, L_LZD_BWD,
    L_HDR_COMPOSE, L_HDR_UPDATE, L_SN_POWER, L_SN_SCALE
};
constexpr size_t LZ_SHMEM = 160 * 1024;   // the long kernels use the whole LDS (avc_long.hip)

// conv_gemm instantiations (avc_gemm_variants.h); the planner autotunes one per
// launch and precision on first use of a workspace.
struct Variant {
    int prec, wm, wn, wgm, wgn, kc;
    const char* name;
    int mt() const { return 32 * wm * wgm; }
    int nt() const { return 32 * wn * wgn; }
    int threads() const { return 64 * wgm * wgn; }
};
static const Variant VARIANTS[] = {
#define AVC_GEMM_VARIANT(I, PREC, WM, WN, WGM, WGN, KC, NAME) {PREC, WM, WN, WGM, WGN, KC, NAME},
#include "avc_gemm_variants.h"
#undef AVC_GEMM_VARIANT
};
constexpr int NVARIANTS = sizeof(VARIANTS) / sizeof(VARIANTS[0]);

struct Launch {
    int kind;
    int variant = 0;             // L_GEMM: index into VARIANTS
    int prec = PREC_F32;         // L_GEMM: operand precision of the MFMAs
    int ksplit = 1;              // L_GEMM: split-K factor (then + a splitk_reduce launch)
    int mode = 0, stride = 1;    // L_GEMM: loader specialisation shared by all its problems
    int maxM = 0, maxN = 0;      // L_GEMM: grid extents over its problems
    int minMpad = 0;             // L_GEMM: smallest A row count (a tile may not read past it)
    dim3 grid, block;
    size_t shmem = 0;
    Problem* dprobs = nullptr;   // device problem table (L_GEMM*)
    int nprob = 0;
    HeadArgs head{};
    FusedArgs fz{};              // L_FZ_* / L_LZ_*: per-utterance SpeakerEncoder pass (prec = PREC_*)
    LongArgs lz{};               // L_LZ_*: the long engine's scratch
    int fz_shape = 8;            // L_FZ_*: kernel shape SH (0 = standard config at T = 128, 16 = standard config
                                 // at 64 < T < 128 (runtime lengths), else 1|2|4|8)
    DecArgs dz{};                // L_DZ_*: per-utterance fused Decoder pass (shape: fz_shape 0 | 8)
    DenseArgs dn{};              // L_DENSE: batched conv_affine layer (or its transpose)
    HdrArgs hd{};                // L_HDR_*: the header optimiser's elementwise ends
    SnArgs sn{};                 // L_SN_*: spectral-norm power iteration / weight rescale
    double flop = 0;             // algorithmic FLOPs of this launch
    std::string name;
};

struct Plan {
    std::vector<Launch> launches;
    std::vector<Problem*> owned;
};

struct Workspace {
    int B = 0, T = 0;
    std::vector<int> Tl;        // T_0..T_n (per conv block input lengths)
    DevBuf xin, adv, vc, ptb, m, v, bank, h0, gbank, gxd, g1, ghx, ghy, gmx, gmy, emb_fwd, org, tgt, grad0;
    std::vector<DevBuf> a1, a2, hb;   // per block
    DevBuf losses, table, scal, slab;
    DevBuf pooled, gpooled;           // fused path: [B][128] time-mean of h_N and its gradient
    DevBuf loss_cur;                  // fused head: [B] per-utterance loss of the current iteration
    unsigned long long* masks = nullptr;   // fused path: ReLU' ballot words [B][mask_words]
    int mask_words = 0;
    bool fused = false;               // this (B, T) runs on the fused family (fused or long engine)
    bool lz = false;                  // ... on the long engine (T > 128, or forced)
    LongArgs lza{};                   // long engine: scratch (images, fp32 streams, ballot masks)
    int iters_cap = 0;
    int* step = nullptr;
    Plan fwd, iter, iter_bf16;
    hipGraphExec_t graph = nullptr, graph_bf16 = nullptr;
    Plan hdr_it[2];                   // header optimiser iteration [prec]
    hipGraphExec_t hdr_graph[2] = {nullptr, nullptr};
    DevBuf hdr, hdr_m, hdr_v, hdr_gx; // header [F*T], its Adam state, d loss / d x [N][F*T]
    bool built = false;
    int gen = 0;                      // ctx-unique id of this workspace's current plans (set on every (re)plan)
    // ragged batch (avc_emb_attack_ragged): utterance b has lens[b] frames; inputs / Adam state are packed
    // [80][lens[b]] blocks; long engine, scratch sized for T = the longest
    bool ragged = false;
    std::vector<int> lens;
    RagUtt* rag = nullptr;            // device [B]: lengths, per-block lengths, packed offsets
    double flop_fwd = 0;              // algorithmic FLOPs of one SpeakerEncoder pass over the batch
    size_t X = 0;                     // floats of one input / state array (B x 80 x T, or the packed sum)
};

}  // namespace

struct VcState;   // ContentEncoder + Decoder of the e2e / fb attacks (avc_vc_host.inc)
static void vc_free(avc_ctx* ctx);

struct avc_ctx {
    VcState* vc = nullptr;
    int device = 0;
    avc_se_cfg cfg{};
    int nb = 0;                         // bank kernels
    std::vector<int> bank_k;
    // packed weights (device)
    std::vector<DevBuf> AtF_bank;       // [K][Mpad]
    DevBuf AtF_in, AtB_in;
    std::vector<DevBuf> AtF_c1, AtF_c2, AtB_c1, AtB_c2;
    DevBuf AtB_bank;
    std::vector<int> kpadB_bank;        // K rows per bank segment in AtB_bank
    std::vector<DevBuf> bias_bank;
    DevBuf bias_in;
    std::vector<DevBuf> bias_c1, bias_c2;
    DevBuf head_Wp, head_WpT, head_bias;
    DevBuf head_Wr, head_WrT;           // se_head_v: row-major dense/output weights and transposes
    DevBuf head_Wr16, head_WrT16;       // ... as bf16 (se_head_v<true>, bf16 mode), 16-byte chunk layout
    bool fused_ok = false;              // config fits the fused per-utterance engine
    int engine = AVC_ENGINE_AUTO;       // avc_set_engine
    std::deque<DevBuf> fz_bufs;         // packed fused-engine A operands (both precisions)
    FusedW fzw[2];                      // [PREC_F32], [PREC_BF16]
    std::map<const float*, void*> bf16_of;   // fp32 A matrix -> its bf16 copy (device)
    hipStream_t stream = nullptr;
    hipEvent_t ev_user = nullptr, ev_done = nullptr;
    // per-call constants (Adam table, scalars) go through this persistent pinned buffer:
    // the copies stay asynchronous, and a later call only waits for them (ev_stage), never
    // for the caller's queued work
    float* stage = nullptr;
    size_t stage_n = 0;
    hipEvent_t ev_stage = nullptr;
    // Workspaces cached by shape: (B, T, engine) -> buffers + plans + captured graphs, most
    // recently used first.  A call at a shape seen before re-plans nothing (real data: a stream of
    // mixed-length utterances, and an adv_tgt embedded at its own length before the attack);
    // the least recently used entry is freed past ws_cap entries.
    std::list<Workspace> wss;
    Workspace* cur = nullptr;           // the workspace of the call in progress
    int ws_cap = 6;
    int gen_next = 0;                   // source of Workspace::gen (unique over the ctx's life)
    long n_ws_builds = 0, n_ws_replans = 0, n_ws_hits = 0, n_graph_captures = 0, n_ws_evictions = 0;
    bool profiling = false;
    std::map<std::string, std::pair<double, double>> prof;   // name -> (total ms, total flop)
    std::map<std::string, long> prof_n;
    double prof_iter_ms = 0;
    int prof_iters = 0;
    std::vector<std::string> prof_names;
};

static int dalloc(DevBuf& b, size_t n) {
    if (b.n >= n && b.p) return 0;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
    if (n == 0) return 0;
    HIPCHK(hipMalloc(&b.p, n * sizeof(float)));
    b.n = n;
    return 0;
}

static void dfree(DevBuf& b) {
    if (b.p) hipFree(b.p);
    b.p = nullptr;
    b.n = 0;
}

// The packers build A^T as [K][Mpad]; the kernels read A row-major [Mpad][Kld]
// (k contiguous, Kld = K rounded up to KALIGN with zero columns) so that a K
// chunk of one output row is one 16-byte-vectorised run in HBM and in LDS.
static std::vector<float> pad_rows(const std::vector<float>& At, int Mpad) {
    const int K = (int)(At.size() / Mpad);
    const int Kld = rup(K, KALIGN);
    std::vector<float> A((size_t)Mpad * Kld, 0.f);
    for (int k = 0; k < K; ++k)
        for (int m = 0; m < Mpad; ++m) A[(size_t)m * Kld + k] = At[(size_t)k * Mpad + m];
    return A;
}

static int upload(DevBuf& b, const std::vector<float>& h) {
    if (dalloc(b, h.size())) return 1;
    HIPCHK(hipMemcpy(b.p, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
    return 0;
}

// a table of plain structs into a float-sized device buffer
template <class T>
static int upload_pod(DevBuf& b, const std::vector<T>& h) {
    static_assert(sizeof(T) % sizeof(float) == 0, "table entries are whole floats");
    if (dalloc(b, h.size() * sizeof(T) / sizeof(float))) return 1;
    if (!h.empty()) HIPCHK(hipMemcpy(b.p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    return 0;
}

// fp32 -> bf16, round to nearest even (weights: finite values)
static uint16_t to_bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

// upload an A matrix in fp32 and in bf16 (the bf16 path's MFMA operand)
static int upload_A(avc_ctx* ctx, DevBuf& b, const std::vector<float>& h) {
    if (upload(b, h)) return 1;
    std::vector<uint16_t> hb(h.size());
    for (size_t i = 0; i < h.size(); ++i) hb[i] = to_bf16(h[i]);
    void* d = nullptr;
    HIPCHK(hipMalloc(&d, hb.size() * 2));
    HIPCHK(hipMemcpy(d, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
    ctx->bf16_of[b.p] = d;
    return 0;
}

static void pads_of(int k, int& pl, int& pr) {   // models.py:23-27
    pl = k / 2;
    pr = (k % 2 == 0) ? k / 2 - 1 : k / 2;
}

// forward A^T: At[ci*k + j][co] = W[co][ci][j]  (rows padded to KC, cols to Mpad)
static std::vector<float> pack_fwd(const HostConv& c, int Mpad, int row_base = 0, int Krows = -1,
                                   std::vector<float>* into = nullptr, int ci_lo = 0, int ci_n = -1) {
    if (ci_n < 0) ci_n = c.ci;
    const int K = Krows < 0 ? rup(ci_n * c.k, KSEG) : Krows;
    std::vector<float> local;
    std::vector<float>& At = into ? *into : local;
    if (!into) At.assign((size_t)K * Mpad, 0.f);
    for (int co = 0; co < c.co; ++co)
        for (int ci = 0; ci < ci_n; ++ci)
            for (int j = 0; j < c.k; ++j)
                At[(size_t)(row_base + ci * c.k + j) * Mpad + co] = c.W[((size_t)co * c.ci + ci_lo + ci) * c.k + j];
    return local;
}

// dgrad A^T: At[co*k + j][ci] = W[co][ci][j]
static void pack_bwd(const HostConv& c, int Mpad, int row_base, std::vector<float>& At) {
    for (int co = 0; co < c.co; ++co)
        for (int ci = 0; ci < c.ci; ++ci)
            for (int j = 0; j < c.k; ++j)
                At[(size_t)(row_base + co * c.k + j) * Mpad + ci] = c.W[((size_t)co * c.ci + ci) * c.k + j];
}

// head fragment packing for v_mfma_f32_16x16x4_f32: A[16mt + (l&15)][4kk + (l>>4)]
static void pack_head(const float* W, int Mo, int Ki, bool transpose, float* dst) {
    const int M = transpose ? Ki : Mo, K = transpose ? Mo : Ki;
    for (int mt = 0; mt < M / 16; ++mt)
        for (int kk = 0; kk < K / 4; ++kk)
            for (int l = 0; l < 64; ++l) {
                const int row = 16 * mt + (l & 15), col = 4 * kk + (l >> 4);
                const float v = transpose ? W[(size_t)col * Ki + row] : W[(size_t)row * Ki + col];
                dst[((size_t)mt * (K / 4) + kk) * 64 + l] = v;
            }
}

static size_t weight_count(const avc_se_cfg& c) {
    size_t n = 0;
    for (int k = c.bank_scale; k <= c.bank_size; k += c.bank_scale)
        n += (size_t)c.c_bank * c.c_in * k + c.c_bank;
    const int cin_cat = c.c_bank * (c.bank_size / c.bank_scale) + c.c_in;
    n += (size_t)c.c_h * cin_cat + c.c_h;
    n += 2 * (size_t)c.n_conv_blocks * ((size_t)c.c_h * c.c_h * c.kernel_size + c.c_h);
    n += 2 * (size_t)c.n_dense_blocks * ((size_t)c.c_h * c.c_h + c.c_h);
    n += (size_t)c.c_out * c.c_h + c.c_out;
    return n;
}

extern "C" size_t avc_se_weight_count(const avc_se_cfg* cfg) { return cfg ? weight_count(*cfg) : 0; }
extern "C" const char* avc_last_error(void) { return g_err.c_str(); }
#ifndef AVC_SRC_HASH
#define AVC_SRC_HASH "unknown"
#endif
// "src=<hash>": __graft_entry__.source_hash() of the sources this library was built from
extern "C" const char* avc_version(void) { return "libavc 0.2 (gfx950) src=" AVC_SRC_HASH; }

static int validate_cfg(const avc_se_cfg& c) {
    if (c.c_in <= 0 || c.c_h <= 0 || c.c_out <= 0 || c.c_bank <= 0) return fail("bad channel counts");
    if (c.bank_scale <= 0 || c.bank_size < c.bank_scale) return fail("bad bank_size/bank_scale");
    if (c.kernel_size <= 0) return fail("bad kernel_size");
    if (c.n_conv_blocks < 0 || c.n_conv_blocks > AVC_MAX_BLOCKS) return fail("n_conv_blocks out of range");
    if (c.n_dense_blocks < 0) return fail("bad n_dense_blocks");
    if (c.c_h % 16 || c.c_out % 16 || c.c_h > 128 || c.c_out > 128)
        return fail("libavc head kernel needs c_h, c_out multiples of 16 and <= 128 (got %d, %d)", c.c_h, c.c_out);
    for (int l = 0; l < c.n_conv_blocks; ++l)
        if (c.subsample[l] < 1) return fail("subsample[%d] < 1", l);
    if (c.act != 0 && c.act != 1) return fail("act must be 0 (relu) or 1 (lrelu)");
    const int S = c.c_h > c.c_out ? c.c_h : c.c_out;
    const size_t lds = (size_t)(2 * c.n_dense_blocks + 5) * S * 16 * sizeof(float);
    if (lds > 160 * 1024) return fail("n_dense_blocks too large for the fused head (%zu B LDS)", lds);
    return 0;
}

// ---------------------------------------------------------------------------------
// fused per-utterance engine: eligibility and A-operand packing (avc_fused.hip)
// ---------------------------------------------------------------------------------
static bool fused_cfg_ok(const avc_se_cfg& c) {
    if (c.c_in != FZ_CIN || c.c_h != FZ_C || c.c_bank != FZ_C || c.c_out != FZ_C) return false;
    if (c.bank_scale != 1 || c.bank_size < 1 || c.bank_size > FZ_MAXNB) return false;
    if (c.kernel_size % 2 == 0 || c.kernel_size > 5) return false;   // dY images carry 2*(ks/2) <= 4 zero rows
    if (c.n_conv_blocks < 1 || c.n_conv_blocks > FZ_MAXBLK) return false;
    for (int l = 0; l < c.n_conv_blocks; ++l)
        if (c.subsample[l] != 1 && c.subsample[l] != 2) return false;
    return true;
}

// Fragment packing: [16-row tile][K step][lane][VE] with lane (r = l&15, q = l>>4)
// holding A[16 mt + r][KS step + VE q + e]; zero outside [M) x [K).
template <typename G>
static int fz_pack(avc_ctx* ctx, int prec, int M, int K, G get, const void*& dst, const float** shadow = nullptr,
                   size_t* count = nullptr) {
    const int KS = prec == PREC_F32 ? 16 : 32, VE = KS / 4;
    const int nmt = cdiv(M, 16), nst = cdiv(K, KS);
    std::vector<float> v((size_t)nmt * nst * 64 * VE, 0.f);
    for (int mt = 0; mt < nmt; ++mt)
        for (int ps = 0; ps < nst; ++ps)
            for (int l = 0; l < 64; ++l)
                for (int e = 0; e < VE; ++e) {
                    const int m = 16 * mt + (l & 15), k = KS * ps + VE * (l >> 4) + e;
                    if (m < M && k < K) v[(((size_t)mt * nst + ps) * 64 + l) * VE + e] = get(m, k);
                }
    if (shadow) {   // the same elements in fp32, same order (spectral norm rescales from it)
        ctx->fz_bufs.emplace_back();
        if (upload(ctx->fz_bufs.back(), v)) return 1;
        *shadow = ctx->fz_bufs.back().p;
    }
    if (count) *count = v.size();
    ctx->fz_bufs.emplace_back();
    DevBuf& b = ctx->fz_bufs.back();
    if (prec == PREC_F32) {
        if (upload(b, v)) return 1;
    } else {
        std::vector<uint16_t> h(v.size());
        for (size_t i = 0; i < v.size(); ++i) h[i] = to_bf16(v[i]);
        HIPCHK(hipMalloc(&b.p, h.size() * 2));
        b.n = h.size() / 2;
        HIPCHK(hipMemcpy(b.p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    }
    dst = b.p;
    return 0;
}

// device bias pointers of one fused encoder (SpeakerEncoder or ContentEncoder)
struct FzBias {
    std::vector<const float*> bank, c1, c2;
    const float* in = nullptr;
};

// A operands of the fused encoder kernels in both precisions into dst[PREC_F32 / PREC_BF16]
// (ctx->fz_bufs owns the device buffers; it is a std::deque, so earlier packs stay put)
static int pack_fused(avc_ctx* ctx, FusedW* dst, const std::vector<HostConv>& bank, const HostConv& inc,
                      const std::vector<HostConv>& c1, const std::vector<HostConv>& c2, const FzBias& fb) {
    const int nb = (int)bank.size(), C = FZ_C, CI = FZ_CIN, ks = c1.empty() ? 1 : c1[0].k, cat = inc.ci;
    const int nblk = (int)c1.size();
    for (int prec = 0; prec < 2; ++prec) {
        FusedW& W = dst[prec];
        int rc = 0;
        for (int kb = 0; kb < nb; ++kb) {
            const HostConv& q = bank[kb];
            const int k = q.k;
            // forward bank: A[co][j*80 + ci] = W[co][ci][j]
            rc |= fz_pack(ctx, prec, C, k * CI, [&](int m, int kk) { return q.W[((size_t)m * CI + kk % CI) * k + kk / CI]; },
                          W.bank[kb]);
            // in_conv, bank block kb: A[co][ci'] = W_in[co][kb*128 + ci']
            rc |= fz_pack(ctx, prec, C, C, [&](int m, int kk) { return inc.W[(size_t)m * cat + kb * C + kk]; }, W.in_b[kb]);
            // in_conv^T, bank block: A[ci'][co] = W_in[co][kb*128 + ci']
            rc |= fz_pack(ctx, prec, C, C, [&](int m, int kk) { return inc.W[(size_t)kk * cat + kb * C + m]; }, W.inT_b[kb]);
            // bank^T: A[ci][j*128 + co] = W[co][ci][j]
            rc |= fz_pack(ctx, prec, CI, k * C, [&](int m, int kk) { return q.W[((size_t)(kk % C) * CI + m) * k + kk / C]; },
                          W.bankT[kb]);
            W.b_bank[kb] = fb.bank[kb];
        }
        rc |= fz_pack(ctx, prec, C, CI, [&](int m, int kk) { return inc.W[(size_t)m * cat + nb * C + kk]; }, W.in_x);
        rc |= fz_pack(ctx, prec, CI, C, [&](int m, int kk) { return inc.W[(size_t)kk * cat + nb * C + m]; }, W.inT_x);
        W.b_in = fb.in;
        for (int l = 0; l < nblk; ++l) {
            for (int which = 0; which < 2; ++which) {
                const HostConv& q = which ? c2[l] : c1[l];
                const void*& f = which ? W.c2[l] : W.c1[l];
                const void*& t = which ? W.c2T[l] : W.c1T[l];
                rc |= fz_pack(ctx, prec, C, ks * C, [&](int m, int kk) { return q.W[((size_t)m * C + kk % C) * ks + kk / C]; }, f);
                rc |= fz_pack(ctx, prec, C, ks * C, [&](int m, int kk) { return q.W[((size_t)(kk % C) * C + m) * ks + kk / C]; }, t);
            }
            W.b_c1[l] = fb.c1[l];
            W.b_c2[l] = fb.c2[l];
        }
        if (rc) return 1;
    }
    return 0;
}

static int set_fused_attrs() {
    // every fused kernel needs more than the default 64 KiB of dynamic LDS
#define AVC_FZ_FNS(SH)                                                                      \
    {(const void*)se_fwd_fused<PREC_F32, SH>, fz_lds_fwd(PREC_F32, 128, 5)},                \
        {(const void*)se_fwd_fused<PREC_BF16, SH>, fz_lds_fwd(PREC_BF16, 128, 5)},   \
        {(const void*)se_bwd_fused<PREC_F32, SH>, fz_lds_bwd(PREC_F32, 128)},                \
        {(const void*)se_bwd_fused<PREC_BF16, SH>, fz_lds_bwd_launch(PREC_BF16, 128, SH, 25 * FZ_MASK_WORDS_PER_LAYER)}
    const std::pair<const void*, int> fns[] = {AVC_FZ_FNS(0), AVC_FZ_FNS(1), AVC_FZ_FNS(2), AVC_FZ_FNS(4),
                                               AVC_FZ_FNS(8), AVC_FZ_FNS(16)};
#undef AVC_FZ_FNS
    for (auto& fn : fns) HIPCHK(hipFuncSetAttribute(fn.first, hipFuncAttributeMaxDynamicSharedMemorySize, fn.second));
    // the persistent emb attack kernel: the larger of its two passes' LDS (the forward's with the fused head)
    const int atk = std::max(std::max(fz_lds_fwd(PREC_BF16, 128, 5), (int)((4 * 6 + 8) * FZ_C * sizeof(float))),
                             fz_lds_bwd_launch(PREC_BF16, 128, 16, 25 * FZ_MASK_WORDS_PER_LAYER));
    HIPCHK(hipFuncSetAttribute((const void*)se_attack_fused<PREC_BF16, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, atk));
    HIPCHK(hipFuncSetAttribute((const void*)se_attack_fused<PREC_BF16, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, atk));
    for (const void* fn : {(const void*)lz_se_fwd<PREC_F32>, (const void*)lz_se_fwd<PREC_BF16>,
                           (const void*)lz_se_bwd<PREC_F32>, (const void*)lz_se_bwd<PREC_BF16>,
                           (const void*)lz_dec_fwd<PREC_F32>, (const void*)lz_dec_fwd<PREC_BF16>,
                           (const void*)lz_dec_bwd<PREC_F32>, (const void*)lz_dec_bwd<PREC_BF16>})
        HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LZ_SHMEM));
    return 0;
}

extern "C" int avc_create(int device, const avc_se_cfg* cfgp, const float* w, size_t n_weights, avc_ctx** out) {
    if (!cfgp || !w || !out) return fail("avc_create: null argument");
    const avc_se_cfg& c = *cfgp;
    if (validate_cfg(c)) return 1;
    if (n_weights != weight_count(c))
        return fail("avc_create: got %zu weights, config needs %zu", n_weights, weight_count(c));
    HIPCHK(hipSetDevice(device));
    avc_ctx* ctx = new avc_ctx();
    ctx->device = device;
    ctx->cfg = c;
    for (int k = c.bank_scale; k <= c.bank_size; k += c.bank_scale) ctx->bank_k.push_back(k);
    ctx->nb = (int)ctx->bank_k.size();
    const int nb = ctx->nb;

    // ---- walk the flat state_dict-ordered weights
    const float* p = w;
    std::vector<HostConv> bank(nb);
    for (int i = 0; i < nb; ++i) {
        bank[i] = {c.c_bank, c.c_in, ctx->bank_k[i], p, nullptr};
        p += (size_t)c.c_bank * c.c_in * ctx->bank_k[i];
        bank[i].b = p;
        p += c.c_bank;
    }
    const int cin_cat = c.c_bank * nb + c.c_in;
    HostConv inc{c.c_h, cin_cat, 1, p, nullptr};
    p += (size_t)c.c_h * cin_cat;
    inc.b = p;
    p += c.c_h;
    std::vector<HostConv> c1(c.n_conv_blocks), c2(c.n_conv_blocks);
    for (int l = 0; l < c.n_conv_blocks; ++l) {
        c1[l] = {c.c_h, c.c_h, c.kernel_size, p, nullptr};
        p += (size_t)c.c_h * c.c_h * c.kernel_size;
        c1[l].b = p;
        p += c.c_h;
    }
    for (int l = 0; l < c.n_conv_blocks; ++l) {
        c2[l] = {c.c_h, c.c_h, c.kernel_size, p, nullptr};
        p += (size_t)c.c_h * c.c_h * c.kernel_size;
        c2[l].b = p;
        p += c.c_h;
    }
    const int nd = c.n_dense_blocks;
    std::vector<const float*> dW(2 * nd), dB(2 * nd);
    for (int l = 0; l < nd; ++l) {   // first_dense_layers
        dW[2 * l] = p;
        p += (size_t)c.c_h * c.c_h;
        dB[2 * l] = p;
        p += c.c_h;
    }
    for (int l = 0; l < nd; ++l) {   // second_dense_layers
        dW[2 * l + 1] = p;
        p += (size_t)c.c_h * c.c_h;
        dB[2 * l + 1] = p;
        p += c.c_h;
    }
    const float* oW = p;
    p += (size_t)c.c_out * c.c_h;
    const float* oB = p;
    p += c.c_out;

    int rc = 0;
    auto up = [&](DevBuf& b, const std::vector<float>& h) { rc |= upload(b, h); };
    auto upA = [&](DevBuf& b, const std::vector<float>& h) { rc |= upload_A(ctx, b, h); };
    auto upv = [&](DevBuf& b, const float* src, size_t n) { up(b, std::vector<float>(src, src + n)); };

    // ---- forward packs
    const int MpadB = rup(c.c_bank, 128);
    ctx->AtF_bank.resize(nb);
    ctx->bias_bank.resize(nb);
    for (int i = 0; i < nb; ++i) {
        upA(ctx->AtF_bank[i], pad_rows(pack_fwd(bank[i], MpadB), MpadB));
        upv(ctx->bias_bank[i], bank[i].b, c.c_bank);
    }
    {
        const int MpadH = rup(c.c_h, 128);
        const int k1 = rup(c.c_bank * nb, KSEG), k2 = rup(c.c_in, KSEG);
        std::vector<float> At((size_t)(k1 + k2) * MpadH, 0.f);
        pack_fwd(inc, MpadH, 0, k1 + k2, &At, 0, c.c_bank * nb);
        pack_fwd(inc, MpadH, k1, k1 + k2, &At, c.c_bank * nb, c.c_in);
        upA(ctx->AtF_in, pad_rows(At, MpadH));
        upv(ctx->bias_in, inc.b, c.c_h);
        // in_conv dgrad: M = cin_cat rows (ci), K = c_h (co): At[co][ci] = W[co][ci]
        const int MpadI = rup(cin_cat, 128);
        std::vector<float> Bt((size_t)rup(c.c_h, KSEG) * MpadI, 0.f);
        pack_bwd(inc, MpadI, 0, Bt);
        upA(ctx->AtB_in, pad_rows(Bt, MpadI));
    }
    ctx->AtF_c1.resize(c.n_conv_blocks);
    ctx->AtF_c2.resize(c.n_conv_blocks);
    ctx->AtB_c1.resize(c.n_conv_blocks);
    ctx->AtB_c2.resize(c.n_conv_blocks);
    ctx->bias_c1.resize(c.n_conv_blocks);
    ctx->bias_c2.resize(c.n_conv_blocks);
    for (int l = 0; l < c.n_conv_blocks; ++l) {
        const int MpadH = rup(c.c_h, 128);
        upA(ctx->AtF_c1[l], pad_rows(pack_fwd(c1[l], MpadH), MpadH));
        upA(ctx->AtF_c2[l], pad_rows(pack_fwd(c2[l], MpadH), MpadH));
        const int Kb = rup(c.c_h * c.kernel_size, KSEG);
        std::vector<float> b1((size_t)Kb * MpadH, 0.f), b2((size_t)Kb * MpadH, 0.f);
        pack_bwd(c1[l], MpadH, 0, b1);
        pack_bwd(c2[l], MpadH, 0, b2);
        upA(ctx->AtB_c1[l], pad_rows(b1, MpadH));
        upA(ctx->AtB_c2[l], pad_rows(b2, MpadH));
        upv(ctx->bias_c1[l], c1[l].b, c.c_h);
        upv(ctx->bias_c2[l], c2[l].b, c.c_h);
    }
    {   // bank dgrad: one GEMM over all bank kernels, M = c_in
        const int MpadX = rup(c.c_in, 128);
        int Ktot = 0;
        for (int i = 0; i < nb; ++i) {
            ctx->kpadB_bank.push_back(rup(c.c_bank * ctx->bank_k[i], KSEG));
            Ktot += ctx->kpadB_bank.back();
        }
        std::vector<float> At((size_t)Ktot * MpadX, 0.f);
        int row = 0;
        for (int i = 0; i < nb; ++i) {
            pack_bwd(bank[i], MpadX, row, At);
            row += ctx->kpadB_bank[i];
        }
        upA(ctx->AtB_bank, pad_rows(At, MpadX));
    }
    {   // head
        const size_t CC = (size_t)c.c_h * c.c_h;
        const size_t tot = 2 * nd * CC + (size_t)c.c_out * c.c_h;
        std::vector<float> Wp(tot), WpT(tot), bias;
        for (int l = 0; l < 2 * nd; ++l) {
            pack_head(dW[l], c.c_h, c.c_h, false, Wp.data() + l * CC);
            pack_head(dW[l], c.c_h, c.c_h, true, WpT.data() + l * CC);
            bias.insert(bias.end(), dB[l], dB[l] + c.c_h);
        }
        pack_head(oW, c.c_out, c.c_h, false, Wp.data() + 2 * nd * CC);
        pack_head(oW, c.c_out, c.c_h, true, WpT.data() + 2 * nd * CC);
        bias.insert(bias.end(), oB, oB + c.c_out);
        up(ctx->head_Wp, Wp);
        up(ctx->head_WpT, WpT);
        up(ctx->head_bias, bias);
        // se_head_v copies: W_l [C][C] then W_out [D][C] and the transposes W_l^T [C][C],
        // W_out^T [C][D], each row permuted so that thread slice q's weights
        // W[m][8i + 2q + e] (i < K/8, e < 2) are the contiguous run [q*K/4, (q+1)*K/4)
        std::vector<float> Wr(tot), WrT(tot);
        auto perm = [](int k, int K) {   // natural column k -> position in the permuted row
            const int i = k / 8, q = (k % 8) / 2, e = k % 2;
            return q * (K / 4) + 2 * i + e;
        };
        for (int l = 0; l < 2 * nd; ++l)
            for (int r = 0; r < c.c_h; ++r)
                for (int k = 0; k < c.c_h; ++k) {
                    Wr[l * CC + (size_t)r * c.c_h + perm(k, c.c_h)] = dW[l][(size_t)r * c.c_h + k];
                    WrT[l * CC + (size_t)k * c.c_h + perm(r, c.c_h)] = dW[l][(size_t)r * c.c_h + k];
                }
        for (int r = 0; r < c.c_out; ++r)
            for (int k = 0; k < c.c_h; ++k) {
                Wr[2 * nd * CC + (size_t)r * c.c_h + perm(k, c.c_h)] = oW[(size_t)r * c.c_h + k];
                WrT[2 * nd * CC + (size_t)k * c.c_out + perm(r, c.c_out)] = oW[(size_t)r * c.c_h + k];
            }
        // lane-interleave for coalesced loads: thread t = 4m + q of se_head_v (wave t/64,
        // lane t%64) reads its 32 permuted weights as 8 f32x4 chunks; chunk e of every lane
        // of a wave is stored contiguously, so each of the 8 load instructions reads one
        // 1 KiB run instead of 16 B from each of 64 different lines
        auto interleave = [&](std::vector<float>& W) {
            if (c.c_h != 128 || c.c_out != 128) return;   // se_head_v's shape (fused engine)
            std::vector<float> o(W.size());
            for (size_t mat = 0; mat < W.size() / (128 * 128); ++mat) {
                const float* src = W.data() + mat * 128 * 128;
                float* dst = o.data() + mat * 128 * 128;
                for (int t = 0; t < 512; ++t)
                    for (int e = 0; e < 8; ++e)
                        for (int j = 0; j < 4; ++j)
                            dst[((size_t)((t / 64) * 8 + e) * 64 + (t % 64)) * 4 + j] = src[(size_t)t * 32 + 4 * e + j];
            }
            W.swap(o);
        };
        // bf16 copies for the bf16 mode: chunk c (8 weights) of thread t at element
        // ((t/64*4 + c)*64 + t%64)*8 of each matrix (one 1 KiB run per load instruction)
        auto to16 = [&](const std::vector<float>& W, DevBuf& dst) {
            if (c.c_h != 128 || c.c_out != 128) return;
            std::vector<uint16_t> o(W.size());
            for (size_t mat = 0; mat < W.size() / (128 * 128); ++mat) {
                const float* src = W.data() + mat * 128 * 128;
                uint16_t* d = o.data() + mat * 128 * 128;
                for (int t = 0; t < 512; ++t)
                    for (int cc = 0; cc < 4; ++cc)
                        for (int i = 0; i < 8; ++i)
                            d[((size_t)((t / 64) * 4 + cc) * 64 + (t % 64)) * 8 + i] = to_bf16(src[(size_t)t * 32 + 8 * cc + i]);
            }
            if (hipMalloc(&dst.p, o.size() * 2) != hipSuccess ||
                hipMemcpy(dst.p, o.data(), o.size() * 2, hipMemcpyHostToDevice) != hipSuccess)
                rc |= fail("avc_create: head bf16 upload failed");
            dst.n = o.size() / 2;
        };
        to16(Wr, ctx->head_Wr16);
        to16(WrT, ctx->head_WrT16);
        interleave(Wr);
        interleave(WrT);
        up(ctx->head_Wr, Wr);
        up(ctx->head_WrT, WrT);
    }
    ctx->fused_ok = fused_cfg_ok(c);
    if (!rc && ctx->fused_ok) {
        FzBias fb;
        for (int i = 0; i < nb; ++i) fb.bank.push_back(ctx->bias_bank[i].p);
        for (int l = 0; l < c.n_conv_blocks; ++l) {
            fb.c1.push_back(ctx->bias_c1[l].p);
            fb.c2.push_back(ctx->bias_c2[l].p);
        }
        fb.in = ctx->bias_in.p;
        rc |= pack_fused(ctx, ctx->fzw, bank, inc, c1, c2, fb);
        rc |= set_fused_attrs();
    }
    if (rc) {
        avc_destroy(ctx);
        return 1;
    }
    hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_user, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_stage, hipEventDisableTiming);
    if (e == hipSuccess) {
        const int S = c.c_h > c.c_out ? c.c_h : c.c_out;
        const size_t lds = (size_t)(2 * nd + 5) * S * 16 * sizeof(float);
        e = hipFuncSetAttribute((const void*)se_head, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    if (e != hipSuccess) {
        avc_destroy(ctx);
        return fail("avc_create: %s", hipGetErrorString(e));
    }
    *out = ctx;
    return 0;
}

static void free_plan(Plan& pl) {
    for (Problem* p : pl.owned) hipFree(p);
    pl.owned.clear();
    pl.launches.clear();
}

static void free_plans(Workspace& ws) {
    if (ws.graph) (void)hipGraphExecDestroy(ws.graph);
    if (ws.graph_bf16) (void)hipGraphExecDestroy(ws.graph_bf16);
    ws.graph = ws.graph_bf16 = nullptr;
    for (int p = 0; p < 2; ++p) {
        if (ws.hdr_graph[p]) (void)hipGraphExecDestroy(ws.hdr_graph[p]);
        ws.hdr_graph[p] = nullptr;
        free_plan(ws.hdr_it[p]);
    }
    free_plan(ws.fwd);
    free_plan(ws.iter);
    free_plan(ws.iter_bf16);
}

static void free_ws(Workspace& ws) {
    free_plans(ws);
    DevBuf* bufs[] = {&ws.xin, &ws.adv, &ws.vc, &ws.ptb, &ws.m, &ws.v, &ws.bank, &ws.h0, &ws.gbank, &ws.gxd,
                      &ws.g1, &ws.ghx, &ws.ghy, &ws.gmx, &ws.gmy, &ws.emb_fwd, &ws.org, &ws.tgt, &ws.grad0, &ws.losses, &ws.table, &ws.scal, &ws.slab, &ws.pooled, &ws.gpooled, &ws.loss_cur,
                      &ws.hdr, &ws.hdr_m, &ws.hdr_v, &ws.hdr_gx};
    for (DevBuf* b : bufs) dfree(*b);
    for (auto& b : ws.a1) dfree(b);
    for (auto& b : ws.a2) dfree(b);
    for (auto& b : ws.hb) dfree(b);
    ws.a1.clear();
    ws.a2.clear();
    ws.hb.clear();
    if (ws.step) hipFree(ws.step);
    ws.step = nullptr;
    if (ws.masks) hipFree(ws.masks);
    ws.masks = nullptr;
    if (ws.lza.img[0]) hipFree(ws.lza.img[0]);
    if (ws.lza.fl[0]) hipFree(ws.lza.fl[0]);
    if (ws.lza.masks) hipFree(ws.lza.masks);
    ws.lza = LongArgs{};
    if (ws.rag) hipFree(ws.rag);
    ws.rag = nullptr;
    ws.ragged = false;
    ws.lens.clear();
    ws.fused = false;
    ws.lz = false;
    ws.built = false;
    ws.B = ws.T = 0;
    ws.iters_cap = 0;
}

extern "C" void avc_destroy(avc_ctx* ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    vc_free(ctx);
    for (Workspace& w : ctx->wss) free_ws(w);
    ctx->wss.clear();
    ctx->cur = nullptr;
    for (auto* v : {&ctx->AtF_bank, &ctx->AtF_c1, &ctx->AtF_c2, &ctx->AtB_c1, &ctx->AtB_c2, &ctx->bias_bank,
                    &ctx->bias_c1, &ctx->bias_c2})
        for (auto& b : *v) dfree(b);
    for (DevBuf* b : {&ctx->AtF_in, &ctx->AtB_in, &ctx->AtB_bank, &ctx->bias_in, &ctx->head_Wp,
                      &ctx->head_WpT, &ctx->head_bias, &ctx->head_Wr, &ctx->head_WrT, &ctx->head_Wr16,
                      &ctx->head_WrT16})
        dfree(*b);
    for (auto& b : ctx->fz_bufs) dfree(b);
    for (auto& kv : ctx->bf16_of) (void)hipFree(kv.second);
    ctx->bf16_of.clear();
    if (ctx->ev_user) hipEventDestroy(ctx->ev_user);
    if (ctx->ev_done) hipEventDestroy(ctx->ev_done);
    if (ctx->ev_stage) hipEventDestroy(ctx->ev_stage);
    if (ctx->stage) (void)hipHostFree(ctx->stage);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
}

// ---------------------------------------------------------------------------------
// planning
// ---------------------------------------------------------------------------------

static Seg make_seg(const float* src, int k0, int C, int c_off, int src_C, int src_T, int ks, int stride, int pl,
                    int pr, int mode) {
    Seg s{};
    s.src = src;
    s.k0 = k0;
    s.kpad = rup(C * ks, KSEG);
    s.C = C;
    s.c_off = c_off;
    s.src_C = src_C;
    s.src_T = src_T;
    s.ks = ks;
    s.stride = stride;
    s.pl = pl;
    s.pr = pr;
    s.mode = mode;
    return s;
}

static Problem base_problem(int M, int Mpad, int N, int T_out, const float* At, const float* bias, int act) {
    Problem p{};
    p.M = M;
    p.Mpad = Mpad;
    p.N = N;
    p.T_out = T_out;
    p.At = At;
    p.bias = bias;
    p.act = act;
    return p;
}

static void add_seg(Problem& p, const Seg& s) {
    p.seg[p.nseg++] = s;
    p.K = s.k0 + s.kpad;
    p.Kld = rup(p.K, KALIGN);
}

static dim3 gemm_grid(const Launch& L, int variant) {
    const Variant& v = VARIANTS[variant];
    return dim3(cdiv(L.maxN, v.nt()), cdiv(L.maxM, v.mt()), L.nprob * L.ksplit);
}

// Split-K factor of a layer.  It may depend on the layer's shape per utterance
// (T_out, K, M) but NOT on the batch size, so that a batch and any shard of it
// sum every output in the same order (bitwise shard invariance); the split
// boundaries are multiples of KALIGN rows, so the tile variant cannot move them.
static int choose_ksplit(const Problem& p, int nprob) {
    if (const char* e = getenv("AVC_KSPLIT")) return std::max(1, std::min(KSPLIT_MAX, atoi(e)));
    if (nprob > 1 || p.M > 128) return 1;
    const int kb = p.K / KALIGN;                 // K in KALIGN blocks
    int ks = 1;
    if (p.K >= 2048) ks = 4;                     // conv-bank dgrad (K = 4608 at the AdaIN-VC config)
    else if (p.T_out <= 32) ks = 4;
    else if (p.T_out <= 64) ks = 2;
    return std::max(1, std::min(ks, kb));
}

// A variant may run a launch only if its M tiles stay inside every A matrix
// (rows up to Mpad are allocated; the kernel reads whole M tiles of A).
static bool variant_fits(const Launch& L, int v) {
    const int mt = VARIANTS[v].mt();
    return VARIANTS[v].prec == L.prec && cdiv(L.maxM, mt) * mt <= L.minMpad;
}

// default tile before autotuning: the largest tile of this precision whose grid
// still has >= 512 workgroups (2 per CU), else the smallest tile
static int default_variant(const Launch& L, const std::vector<Problem>& ps, int prec) {
    int best = -1, small = -1;
    long best_area = 0, small_area = 1L << 40;
    for (int v = 0; v < NVARIANTS; ++v) {
        if (VARIANTS[v].prec != prec || !variant_fits(L, v)) continue;
        const long area = (long)VARIANTS[v].mt() * VARIANTS[v].nt();
        long wgs = 0;
        for (auto& p : ps) wgs += (long)cdiv(p.M, VARIANTS[v].mt()) * cdiv(p.N, VARIANTS[v].nt());
        if (wgs >= 512 && area > best_area) {
            best = v;
            best_area = area;
        }
        if (area < small_area) {
            small = v;
            small_area = area;
        }
    }
    return best >= 0 ? best : small;
}

static int add_gemm(avc_ctx* ctx, Plan& pl, std::vector<Problem> ps, double flop, const std::string& what,
                    int prec) {
    int gx = 0, gy = 0, minMpad = 0;
    const int ksplit_req = choose_ksplit(ps[0], (int)ps.size());
    int ksplit = 1;
    if (ksplit_req > 1) {
        Problem& p = ps[0];
        p.ksplit_rows = rup(cdiv(p.K, ksplit_req), KALIGN);
        ksplit = cdiv(p.K, p.ksplit_rows);
        if (ksplit > 1) {
            if ((size_t)ksplit * p.M * p.N > ctx->cur->slab.n) return fail("internal: split-K slab too small");
            p.slab = ctx->cur->slab.p;
        } else {
            p.ksplit_rows = 0;
        }
    }
    for (auto& p : ps) {
        auto it = ctx->bf16_of.find(p.At);
        if (it == ctx->bf16_of.end()) return fail("internal: no bf16 copy of an A matrix");
        p.Ab = it->second;
        for (int i = 0; i < p.nseg; ++i)
            if (p.seg[i].mode != ps[0].seg[0].mode || p.seg[i].stride != ps[0].seg[0].stride)
                return fail("internal: mixed loader modes in one launch");
        if (p.K % KSEG) return fail("internal: K %d not a multiple of %d", p.K, KSEG);
        if (p.Mpad % 128) return fail("internal: Mpad %d not a multiple of 128", p.Mpad);
        if (p.Kld != rup(p.K, KALIGN)) return fail("internal: Kld %d for K %d", p.Kld, p.K);
        gx = std::max(gx, p.N);
        gy = std::max(gy, p.M);
        minMpad = minMpad ? std::min(minMpad, p.Mpad) : p.Mpad;
    }
    Problem* d = nullptr;
    HIPCHK(hipMalloc(&d, ps.size() * sizeof(Problem)));
    HIPCHK(hipMemcpy(d, ps.data(), ps.size() * sizeof(Problem), hipMemcpyHostToDevice));
    pl.owned.push_back(d);
    Launch L;
    L.kind = L_GEMM;
    L.prec = prec;
    L.ksplit = ksplit;
    L.maxN = gx;
    L.maxM = gy;
    L.minMpad = minMpad;
    L.variant = default_variant(L, ps, prec);
    if (L.variant < 0) return fail("internal: no GEMM variant fits %s", what.c_str());
    L.mode = ps[0].seg[0].mode;
    L.stride = ps[0].seg[0].stride;
    L.block = dim3(256);
    L.dprobs = d;
    L.nprob = (int)ps.size();
    L.flop = flop;
    L.name = what;
    pl.launches.push_back(L);
    return 0;
}

// SpeakerEncoder forward (models.py:327-343) from `x` up to h_N, then the head.
static int plan_forward(avc_ctx* ctx, Workspace& ws, Plan& pl, const float* x, bool attack, int prec) {
    const avc_se_cfg& c = ctx->cfg;
    const int B = ws.B, T = ws.T, nb = ctx->nb;
    const int N0 = B * T;
    {   // conv bank: nb problems in one launch
        std::vector<Problem> ps;
        double flop = 0;
        for (int i = 0; i < nb; ++i) {
            const int k = ctx->bank_k[i];
            int pl_, pr_;
            pads_of(k, pl_, pr_);
            Problem p = base_problem(c.c_bank, rup(c.c_bank, 128), N0, T, ctx->AtF_bank[i].p, ctx->bias_bank[i].p,
                                     c.act);
            add_seg(p, make_seg(x, 0, c.c_in, 0, c.c_in, T, k, 1, pl_, pr_, SEG_FWD));
            p.epi = EPI_ACT;
            p.out0 = ws.bank.p;
            p.out0_C = nb * c.c_bank;
            p.out0_coff = i * c.c_bank;
            if (attack && i == 0) p.tick = ws.step;
            ps.push_back(p);
            flop += 2.0 * c.c_bank * c.c_in * k * N0;
        }
        if (add_gemm(ctx, pl, ps, flop, "bank", prec)) return 1;
    }
    {   // in_conv_layer over cat(bank, x) (models.py:103,337-338)
        Problem p = base_problem(c.c_h, rup(c.c_h, 128), N0, T, ctx->AtF_in.p, ctx->bias_in.p, c.act);
        add_seg(p, make_seg(ws.bank.p, 0, nb * c.c_bank, 0, nb * c.c_bank, T, 1, 1, 0, 0, SEG_FWD));
        add_seg(p, make_seg(x, p.K, c.c_in, 0, c.c_in, T, 1, 1, 0, 0, SEG_FWD));
        p.epi = EPI_ACT;
        p.out0 = ws.h0.p;
        p.out0_C = c.c_h;
        if (add_gemm(ctx, pl, {p}, 2.0 * c.c_h * (nb * c.c_bank + c.c_in) * N0, "in_conv", prec)) return 1;
    }
    int kpl, kpr;
    pads_of(c.kernel_size, kpl, kpr);
    for (int l = 0; l < c.n_conv_blocks; ++l) {
        const int Ti = ws.Tl[l], To = ws.Tl[l + 1], s = c.subsample[l];
        const float* hin = l == 0 ? ws.h0.p : ws.hb[l - 1].p;
        Problem p1 = base_problem(c.c_h, rup(c.c_h, 128), B * Ti, Ti, ctx->AtF_c1[l].p, ctx->bias_c1[l].p, c.act);
        add_seg(p1, make_seg(hin, 0, c.c_h, 0, c.c_h, Ti, c.kernel_size, 1, kpl, kpr, SEG_FWD));
        p1.epi = EPI_ACT;
        p1.out0 = ws.a1[l].p;
        p1.out0_C = c.c_h;
        if (add_gemm(ctx, pl, {p1}, 2.0 * c.c_h * c.c_h * c.kernel_size * B * Ti, "conv1.b" + std::to_string(l), prec)) return 1;
        Problem p2 = base_problem(c.c_h, rup(c.c_h, 128), B * To, To, ctx->AtF_c2[l].p, ctx->bias_c2[l].p, c.act);
        add_seg(p2, make_seg(ws.a1[l].p, 0, c.c_h, 0, c.c_h, Ti, c.kernel_size, s, kpl, kpr, SEG_FWD));
        p2.epi = EPI_BLOCK;
        p2.out0 = ws.a2[l].p;
        p2.out0_C = c.c_h;
        p2.out1 = ws.hb[l].p;
        p2.out1_C = c.c_h;
        p2.aux0 = hin;
        p2.aux0_C = c.c_h;
        p2.aux0_T = Ti;
        p2.pool_s = s;
        if (add_gemm(ctx, pl, {p2}, 2.0 * c.c_h * c.c_h * c.kernel_size * B * To, "conv2.b" + std::to_string(l), prec)) return 1;
    }
    {   // head
        Launch L;
        L.kind = L_HEAD;
        L.grid = dim3(cdiv(B, 16));
        L.block = dim3(512);
        const int S = std::max(c.c_h, c.c_out);
        L.shmem = (size_t)(2 * c.n_dense_blocks + 5) * S * 16 * sizeof(float);
        HeadArgs& A = L.head;
        A.hN = c.n_conv_blocks ? ws.hb[c.n_conv_blocks - 1].p : ws.h0.p;
        A.g_hN = ws.ghx.p;
        A.g_hN_masked = ws.gmx.p;   // dY of the last block's conv2 dgrad: g * act'(a2_last)
        A.mask_hN = c.n_conv_blocks ? ws.a2[c.n_conv_blocks - 1].p : ws.h0.p;
        A.Wp = ctx->head_Wp.p;
        A.WpT = ctx->head_WpT.p;
        A.bias = ctx->head_bias.p;
        A.emb_out = ws.emb_fwd.p;
        A.tgt = ws.tgt.p;
        A.org = ws.org.p;
        A.losses = ws.losses.p;
        A.step = ws.step;
        A.B = B;
        A.C = c.c_h;
        A.TN = ws.Tl[c.n_conv_blocks];
        A.D = c.c_out;
        A.n_dense = c.n_dense_blocks;
        A.act = c.act;
        A.mode = attack ? 1 : 0;
        A.scal = ws.scal.p;
        A.loss_len = ws.iters_cap;
        const double dense = 2.0 * c.c_h * c.c_h * 2 * c.n_dense_blocks + 2.0 * c.c_out * c.c_h;
        L.flop = dense * B * (attack ? 2 : 1);
        L.name = "se_head";
        pl.launches.push_back(L);
    }
    return 0;
}

// Input-gradient of the SpeakerEncoder back to the perturbation + Adam (fused).
static int plan_backward(avc_ctx* ctx, Workspace& ws, Plan& pl, int prec) {
    const avc_se_cfg& c = ctx->cfg;
    const int B = ws.B, T = ws.T, nb = ctx->nb;
    int kpl, kpr;
    pads_of(c.kernel_size, kpl, kpr);
    // g(h_l) ping-pong (unmasked: feeds the residual avg-pool^T) and its ReLU'-masked
    // copy (the dY of the next dgrad).  The head wrote g(h_N) -> ghx, masked -> gmx.
    DevBuf* gcur = &ws.ghx;
    DevBuf* gnext = &ws.ghy;
    DevBuf* mcur = &ws.gmx;
    DevBuf* mnext = &ws.gmy;
    const int MpadH = rup(c.c_h, 128);
    for (int l = c.n_conv_blocks - 1; l >= 0; --l) {
        const int Ti = ws.Tl[l], To = ws.Tl[l + 1], s = c.subsample[l];
        // conv2^T: dY = g(h_{l+1}) * act'(a2_l) (masked by its producer), stride s; * act'(a1_l)
        Problem p2 = base_problem(c.c_h, MpadH, B * Ti, Ti, ctx->AtB_c2[l].p, nullptr, c.act);
        add_seg(p2, make_seg(mcur->p, 0, c.c_h, 0, c.c_h, To, c.kernel_size, s, kpl, kpr, SEG_BWD));
        p2.both_edges = Ti <= kpl + kpr + 1;
        p2.epi = EPI_MASK;
        p2.out0 = ws.g1.p;
        p2.out0_C = c.c_h;
        p2.aux0 = ws.a1[l].p;
        p2.aux0_C = c.c_h;
        p2.aux0_T = Ti;
        if (add_gemm(ctx, pl, {p2}, 2.0 * c.c_h * c.c_h * c.kernel_size * B * To, "conv2_dgrad.b" + std::to_string(l), prec)) return 1;
        // conv1^T + residual avg-pool^T -> g(h_l), and its copy masked by the ReLU that
        // produced h_l (a2_{l-1}, or h0's in_conv ReLU for l = 0)
        Problem p1 = base_problem(c.c_h, MpadH, B * Ti, Ti, ctx->AtB_c1[l].p, nullptr, c.act);
        add_seg(p1, make_seg(ws.g1.p, 0, c.c_h, 0, c.c_h, Ti, c.kernel_size, 1, kpl, kpr, SEG_BWD));
        p1.both_edges = Ti <= kpl + kpr + 1;
        p1.epi = EPI_POOLT;
        p1.out0 = l > 0 ? gnext->p : nullptr;
        p1.out0_C = c.c_h;
        p1.out1 = mnext->p;
        p1.out1_C = c.c_h;
        p1.aux1 = l > 0 ? ws.a2[l - 1].p : ws.h0.p;
        p1.aux0 = gcur->p;
        p1.aux0_C = c.c_h;
        p1.aux0_T = To;
        p1.pool_s = s;
        if (add_gemm(ctx, pl, {p1}, 2.0 * c.c_h * c.c_h * c.kernel_size * B * Ti, "conv1_dgrad.b" + std::to_string(l), prec)) return 1;
        std::swap(gcur, gnext);
        std::swap(mcur, mnext);
    }
    const int N0 = B * T;
    const int cin_cat = nb * c.c_bank + c.c_in;
    {   // in_conv^T: rows = cat channels; dY = g(h0) * act'(h0)
        Problem p = base_problem(cin_cat, rup(cin_cat, 128), N0, T, ctx->AtB_in.p, nullptr, c.act);
        add_seg(p, make_seg(mcur->p, 0, c.c_h, 0, c.c_h, T, 1, 1, 0, 0, SEG_BWD));
        p.epi = EPI_INCONV_T;
        p.split = nb * c.c_bank;
        p.out0 = ws.gbank.p;
        p.out0_C = nb * c.c_bank;
        p.out1 = ws.gxd.p;
        p.out1_C = c.c_in;
        p.aux0 = ws.bank.p;
        p.aux0_C = nb * c.c_bank;
        p.aux0_T = T;
        if (add_gemm(ctx, pl, {p}, 2.0 * c.c_h * cin_cat * N0, "in_conv_dgrad", prec)) return 1;
    }
    {   // conv bank^T over all kernels + x passthrough + tanh' + Adam
        Problem p = base_problem(c.c_in, rup(c.c_in, 128), N0, T, ctx->AtB_bank.p, nullptr, c.act);
        double flop = 0;
        int k0 = 0;
        for (int i = 0; i < nb; ++i) {
            const int k = ctx->bank_k[i];
            int pl_, pr_;
            pads_of(k, pl_, pr_);
            add_seg(p, make_seg(ws.gbank.p, k0, c.c_bank, i * c.c_bank, nb * c.c_bank, T, k, 1, pl_, pr_,
                                SEG_BWD));
            k0 += ctx->kpadB_bank[i];
            flop += 2.0 * c.c_bank * c.c_in * k * N0;
            if (T <= pl_ + pr_ + 1) p.both_edges = 1;
        }
        if (nb > MAX_SEGS) return fail("bank_size/bank_scale > %d kernels not supported", MAX_SEGS);
        p.epi = EPI_ADAM;
        p.aux0 = ws.gxd.p;
        p.step = ws.step;
        p.scal = ws.scal.p;
        p.table_len = ws.iters_cap;
        AdamArgs& A = p.adam;
        A.ptb = ws.ptb.p;
        A.m = ws.m.p;
        A.v = ws.v.p;
        A.vc = ws.vc.p;
        A.adv = ws.adv.p;
        A.table = ws.table.p;
        A.grad0 = ws.grad0.p;
        A.b1c = (float)(1.0 - 0.9);
        A.b2 = 0.999f;
        A.b2c = (float)(1.0 - 0.999);
        A.adam_eps = 1e-8f;
        if (add_gemm(ctx, pl, {p}, flop, "bank_dgrad_adam", prec)) return 1;
    }
    return 0;
}

// ---------------------------------------------------------------------------------
// fused per-utterance plans: [se_fwd_fused] -> se_head (batched) [-> se_bwd_fused]
// ---------------------------------------------------------------------------------
static double fz_fwd_flop(const avc_se_cfg& c, const std::vector<int>& Tl, const std::vector<int>& bank_k) {
    double mac = 0;
    const int T = Tl[0];
    for (int k : bank_k) mac += (double)c.c_bank * c.c_in * k * T;
    mac += (double)c.c_h * (c.c_bank * (int)bank_k.size() + c.c_in) * T;
    for (int l = 0; l < c.n_conv_blocks; ++l)
        mac += (double)c.c_h * c.c_h * c.kernel_size * (Tl[l] + Tl[l + 1]);
    return 2.0 * mac;
}

static FusedArgs fused_args(avc_ctx* ctx, Workspace& ws, int prec) {
    const avc_se_cfg& c = ctx->cfg;
    FusedArgs A{};
    A.B = ws.B;
    A.T = ws.T;
    A.nb = ctx->nb;
    A.ks = c.kernel_size;
    A.nblk = c.n_conv_blocks;
    A.act = c.act;
    for (int l = 0; l < c.n_conv_blocks; ++l) A.sub[l] = c.subsample[l];
    for (int l = 0; l <= c.n_conv_blocks; ++l) A.Tl[l] = ws.Tl[l];
    A.mask_words = ws.mask_words;
    A.masks = ws.masks;
    A.pooled = ws.pooled.p;
    A.g_pooled = ws.gpooled.p;
    A.step = ws.step;
    A.scal = ws.scal.p;
    A.table_len = ws.iters_cap;
    A.w = ctx->fzw[prec];
    A.rag = ws.rag;
    return A;
}

// fused kernel shape: 0 = AdaIN-VC config.yaml defaults at T = 128 (every layer shape
// compile-time), else the fragment bound 1|2|4|8 >= ceil(T/16)
static int fused_shape(avc_ctx* ctx, int T) {
    const avc_se_cfg& c = ctx->cfg;
    bool std_cfg = T == 128 && ctx->nb == 8 && c.kernel_size == 5 && c.n_conv_blocks == 6 && c.act == 0;
    for (int l = 0; std_cfg && l < 6; ++l)
        if (c.subsample[l] != ((l & 1) ? 2 : 1)) std_cfg = false;
    const char* e = getenv("AVC_FUSED_STD");
    const char* rf = getenv("AVC_FUSED_RT_FORCE");   // A/B runs: the runtime-length kernels at T = 128 too
    if (std_cfg && rf && rf[0] == '1') return 16;
    if (std_cfg && !(e && e[0] == '0')) return 0;
    // the standard config at 64 < T < 128: the standard kernels' fragment classes with runtime lengths
    bool std_rt = T > 64 && T < 128 && ctx->nb == 8 && c.kernel_size == 5 && c.n_conv_blocks == 6 && c.act == 0;
    for (int l = 0; std_rt && l < 6; ++l)
        if (c.subsample[l] != ((l & 1) ? 2 : 1)) std_rt = false;
    const char* r = getenv("AVC_FUSED_RT");
    if (std_rt && !(e && e[0] == '0') && !(r && r[0] == '0')) return 16;
    const int nf = cdiv(T, 16);
    return nf <= 1 ? 1 : nf <= 2 ? 2 : nf <= 4 ? 4 : 8;
}

static int plan_fused_forward(avc_ctx* ctx, Workspace& ws, Plan& pl, const float* x, bool attack, int prec) {
    const avc_se_cfg& c = ctx->cfg;
    const int B = ws.B;
    Launch F;
    F.kind = ws.lz ? L_LZ_FWD : L_FZ_FWD;
    F.prec = prec;
    F.grid = dim3(B);
    F.block = dim3(256);
    F.shmem = ws.lz ? LZ_SHMEM : fz_lds_fwd(prec, ws.T, c.kernel_size);
    F.fz = fused_args(ctx, ws, prec);
    F.lz = ws.lza;
    F.fz.x = x;
    F.fz.write_masks = attack ? 1 : 0;
    F.fz.tick = attack ? ws.step : nullptr;
    F.fz_shape = ws.ragged ? 16 : fused_shape(ctx, ws.T);
    F.flop = ws.flop_fwd;
    F.name = prec == PREC_F32 ? "se_fwd_fused<f32>" : "se_fwd_fused<bf16>";
    if (ws.lz) F.name = prec == PREC_F32 ? "lz_se_fwd<f32>" : "lz_se_fwd<bf16>";

    Launch L;
    L.kind = L_HEAD_V;
    L.grid = dim3(cdiv(B, 2));
    L.block = dim3(512);
    const int S = std::max(c.c_h, c.c_out);
    L.shmem = (size_t)(2 * c.n_dense_blocks + 5) * S * 2 * sizeof(float) +
              (size_t)(2 * c.n_dense_blocks * c.c_h + c.c_out + 4 * c.c_out + 2) * sizeof(float);
    HeadArgs& A = L.head;
    L.prec = prec;
    A.Wr = ctx->head_Wr.p;
    A.WrT = ctx->head_WrT.p;
    A.Wr16 = reinterpret_cast<const uint16_t*>(ctx->head_Wr16.p);
    A.WrT16 = reinterpret_cast<const uint16_t*>(ctx->head_WrT16.p);
    A.pooled_in = ws.pooled.p;
    A.g_pooled = attack ? ws.gpooled.p : nullptr;
    A.Wp = ctx->head_Wp.p;
    A.WpT = ctx->head_WpT.p;
    A.bias = ctx->head_bias.p;
    A.emb_out = ws.emb_fwd.p;
    A.tgt = ws.tgt.p;
    A.org = ws.org.p;
    A.losses = ws.losses.p;
    A.step = ws.step;
    A.B = B;
    A.C = c.c_h;
    A.TN = ws.Tl[c.n_conv_blocks];
    A.D = c.c_out;
    A.n_dense = c.n_dense_blocks;
    A.act = c.act;
    A.mode = attack ? 1 : 0;
    A.scal = ws.scal.p;
    A.loss_len = ws.iters_cap;
    const double dense = 2.0 * c.c_h * c.c_h * 2 * c.n_dense_blocks + 2.0 * c.c_out * c.c_h;
    L.flop = dense * B * (attack ? 2 : 1);
    L.name = "se_head_v";

    // emb attack in bf16: the head runs in the forward's tail (se_head_fused), one launch
    // fewer per iteration; AVC_FUSE_HEAD=0 keeps the separate se_head_v launch (A/B runs)
    const char* fe = getenv("AVC_FUSE_HEAD");
    // (standard shape only: the in-kernel chain is unrolled for its n_dense = 6)
    if (attack && prec == PREC_BF16 && ctx->head_Wr16.p && c.c_h == FZ_C && c.c_out == FZ_C && !ws.lz && (F.fz_shape == 0 || F.fz_shape == 16) &&
        c.n_dense_blocks == 6 && !(fe && fe[0] == '0')) {
        const size_t head_lds = (size_t)(4 * c.n_dense_blocks + 8) * FZ_C * sizeof(float);
        F.shmem = std::max(F.shmem, head_lds);
        F.fz.fuse_head = 1;
        F.fz.head = A;
        F.fz.loss_cur = ws.loss_cur.p;
        F.flop += L.flop;
        F.name = "se_fwd_fused<bf16>";
        pl.launches.push_back(F);
        return 0;
    }
    pl.launches.push_back(F);
    pl.launches.push_back(L);
    return 0;
}

static int plan_fused_backward(avc_ctx* ctx, Workspace& ws, Plan& pl, int prec) {
    Launch L;
    L.kind = ws.lz ? L_LZ_BWD : L_FZ_BWD;
    L.prec = prec;
    L.grid = dim3(ws.B);
    L.block = dim3(256);
    L.fz = fused_args(ctx, ws, prec);
    L.lz = ws.lza;
    L.fz_shape = ws.ragged ? 16 : fused_shape(ctx, ws.T);
    // (SH = 16: the LDS images are laid out for the 128-frame bound)
    L.shmem = ws.lz ? LZ_SHMEM : fz_lds_bwd_launch(prec, L.fz_shape == 16 ? 128 : ws.T, L.fz_shape, L.fz.mask_words);
    AdamArgs& A = L.fz.adam;
    A.ptb = ws.ptb.p;
    A.m = ws.m.p;
    A.v = ws.v.p;
    A.vc = ws.vc.p;
    A.adv = ws.adv.p;
    A.table = ws.table.p;
    A.grad0 = ws.grad0.p;
    A.b1c = (float)(1.0 - 0.9);
    A.b2 = 0.999f;
    A.b2c = (float)(1.0 - 0.999);
    A.adam_eps = 1e-8f;
    L.flop = ws.flop_fwd;   // input-gradient only
    L.name = prec == PREC_F32 ? "se_bwd_fused<f32>" : "se_bwd_fused<bf16>";
    if (ws.lz) L.name = prec == PREC_F32 ? "lz_se_bwd<f32>" : "lz_se_bwd<bf16>";
    pl.launches.push_back(L);
    return 0;
}

static int plan_iteration(avc_ctx* ctx, Workspace& ws, Plan& pl, int prec) {
    if (ws.fused)
    {
        if (plan_fused_forward(ctx, ws, pl, ws.adv.p, true, prec) || plan_fused_backward(ctx, ws, pl, prec)) return 1;
        // a forward with the head fused hands its per-utterance loss to the backward, which
        // knows the step (the forward's block 0 advances the counter while it runs)
        const Launch& F = pl.launches[pl.launches.size() - 2];
        if (F.kind == L_FZ_FWD && F.fz.fuse_head) {
            Launch& Bk = pl.launches.back();
            Bk.fz.loss_cur = ws.loss_cur.p;
            Bk.fz.losses = ws.losses.p;
            Bk.fz.loss_len = ws.iters_cap;
        }
        return 0;
    }
    return plan_forward(ctx, ws, pl, ws.adv.p, true, prec) || plan_backward(ctx, ws, pl, prec);
}

static int autotune(avc_ctx* ctx, Plan& pl);

// Engine of a call with T frames: the fused engine up to 128 frames, the long engine above
// (same kernels family, activations chunked through global scratch), the layered engine for
// configs neither is built for.  AVC_FUSED=0 (AUTO only) forces layered, AVC_LONG=1 long.
static int engine_for(avc_ctx* ctx, int T) {
    if (ctx->engine == AVC_ENGINE_LAYERED || !ctx->fused_ok) return AVC_ENGINE_LAYERED;
    const char* fe = getenv("AVC_FUSED");
    if (ctx->engine == AVC_ENGINE_AUTO && fe && fe[0] == '0') return AVC_ENGINE_LAYERED;
    const char* le = getenv("AVC_LONG");
    if (ctx->engine == AVC_ENGINE_LONG || (le && le[0] == '1')) return AVC_ENGINE_LONG;
    return T <= 128 ? AVC_ENGINE_FUSED : AVC_ENGINE_LONG;
}
static bool want_fused(avc_ctx* ctx, int T) { return engine_for(ctx, T) != AVC_ENGINE_LAYERED; }

// long-engine scratch for B utterances of up to T frames and `nlayers` masked layers
static int alloc_long(LongArgs& L, int B, int T, int nlayers) {
    // pad rows around the frames, + LZ_ZR for the decoder's out_conv^T dY image (zeroed over
    // Tn + 3 LZ_ZR rows).  Every stage of a chunk window is clipped to these rows in the kernels
    // (avc_long.hip LzPipe::rows / lz_stage_cap): a stride-2 window spans 2 * 127 + k + 2 rows whatever
    // the layer's length, which read past a short utterance's image (round 3: T <= 178)
    const int rows = T + 3 * LZ_ZR + 16;
    L.img_stride = (int64_t)rows * 128 * 4;                 // fp32-sized rows serve both precisions
    L.fl_stride = (int64_t)((T + 32 + 15) / 16 + LZ_FL_EXTRA) * 4 * 2 * 64 * 4;
    L.nFmax = (T + 15) / 16;
    L.mask_stride = (int64_t)nlayers * L.nFmax * 32;
    // each allocation is recorded in L at once, so free_ws releases a partial set on failure
    char* img = nullptr;
    float* fl = nullptr;
    unsigned long long* mk = nullptr;
    HIPCHK(hipMalloc(&img, 3 * (size_t)B * L.img_stride));
    L.img[0] = img;
    HIPCHK(hipMalloc(&fl, 3 * (size_t)B * L.fl_stride * sizeof(float)));
    L.fl[0] = fl;
    HIPCHK(hipMalloc(&mk, (size_t)B * L.mask_stride * sizeof(unsigned long long)));
    L.masks = mk;
    // every byte a kernel may stage is finite from the start (weights past K are zero, and
    // 0 * NaN would not be)
    HIPCHK(hipMemset(img, 0, 3 * (size_t)B * L.img_stride));
    HIPCHK(hipMemset(fl, 0, 3 * (size_t)B * L.fl_stride * sizeof(float)));
    HIPCHK(hipMemset(mk, 0, (size_t)B * L.mask_stride * sizeof(unsigned long long)));
    for (int i = 0; i < 3; ++i) {
        L.img[i] = img + (size_t)i * B * L.img_stride;
        L.fl[i] = fl + (size_t)i * B * L.fl_stride;
    }
    return 0;
}

// a workspace whose build failed part-way: release what it holds and forget it (returns 1)
static int drop_ws(avc_ctx* ctx);
// HIPCHK for a workspace under construction: on failure the half-built entry is dropped (drop_ws)
#define WSCHK(expr)                                                                                   \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) {                                                                   \
            fail("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__);      \
            return drop_ws(ctx);                                                                  \
        }                                                                                         \
    } while (0)
static int drop_ws(avc_ctx* ctx) {
    for (auto it = ctx->wss.begin(); it != ctx->wss.end(); ++it)
        if (&*it == ctx->cur) {
            (void)hipStreamSynchronize(ctx->stream);
            free_ws(*it);
            ctx->wss.erase(it);
            break;
        }
    ctx->cur = nullptr;
    return 1;
}

// lengths through the conv blocks for T input frames + reflect-pad validity (torch: pad < input length)
static int enc_block_lengths(avc_ctx* ctx, int T, std::vector<int>& Tl) {
    const avc_se_cfg& c = ctx->cfg;
    Tl.assign(1, T);
    int maxpad = 0;
    for (int k : ctx->bank_k) {
        int a, b;
        pads_of(k, a, b);
        maxpad = std::max(maxpad, std::max(a, b));
    }
    if (T <= maxpad) return fail("T=%d too short for the conv bank reflect padding (%d)", T, maxpad);
    int kpl, kpr;
    pads_of(c.kernel_size, kpl, kpr);
    for (int l = 0; l < c.n_conv_blocks; ++l) {
        if (Tl.back() <= std::max(kpl, kpr))
            return fail("T=%d too short: conv block %d input has %d frames (reflect pad %d)", T, l, Tl.back(),
                        std::max(kpl, kpr));
        const int s = c.subsample[l];
        const int To = (Tl.back() + kpl + kpr - c.kernel_size) / s + 1;
        const int Tp = cdiv(Tl.back(), s);
        if (To != Tp) return fail("conv/pool length mismatch at block %d (%d vs %d)", l, To, Tp);
        Tl.push_back(To);
    }
    return 0;
}

// The workspace of a call: B utterances of T frames, or (lens non-null) a ragged batch of B utterances
// of lens[b] frames (long engine; T is ignored).  Cached by shape, most recently used first.
static int ensure_ws(avc_ctx* ctx, int B, int T, int n_iters, const std::vector<int>* lens = nullptr) {
    const avc_se_cfg& c = ctx->cfg;
    if (B <= 0) return fail("batch size must be positive (got %d)", B);
    std::vector<int> Tl;
    std::vector<std::vector<int>> Tls;
    double flop = 0;
    size_t X = 0;
    bool rag_fused = false;
    if (lens) {
        if ((int)lens->size() != B) return fail("ragged batch: %zu lengths for B=%d", lens->size(), B);
        if (!ctx->fused_ok || ctx->engine == AVC_ENGINE_LAYERED)
            return fail("ragged batches run on the long engine (fused-capable config, engine not layered)");
        T = *std::max_element(lens->begin(), lens->end());
        // every length in (64, 128] of the standard config: the fused runtime-length kernels with a
        // per-workgroup length (LDS images laid out for 128 frames); otherwise the long engine
        const int Tmin = *std::min_element(lens->begin(), lens->end());
        const char* rf = getenv("AVC_RAGGED_FUSED");
        rag_fused = Tmin > 64 && T <= 128 && ctx->engine != AVC_ENGINE_LONG && !(rf && rf[0] == '0') &&
                    fused_shape(ctx, 100) == 16 && !(getenv("AVC_LONG") && getenv("AVC_LONG")[0] == '1');
        for (int b = 0; b < B; ++b) {
            std::vector<int> t;
            if (enc_block_lengths(ctx, (*lens)[b], t)) return 1;
            flop += fz_fwd_flop(c, t, ctx->bank_k);
            X += (size_t)c.c_in * (*lens)[b];
            Tls.push_back(t);
        }
    }
    if (rag_fused) T = 128;   // the workspace's bound (LDS layout, mask words); lengths come from ws.rag
    if (enc_block_lengths(ctx, T, Tl)) return 1;
    if (!lens) {
        flop = fz_fwd_flop(c, Tl, ctx->bank_k) * B;
        X = (size_t)B * c.c_in * T;
    }
    const int eng = lens ? (rag_fused ? AVC_ENGINE_FUSED : AVC_ENGINE_LONG) : engine_for(ctx, T);
    const bool fused = eng != AVC_ENGINE_LAYERED, lz = eng == AVC_ENGINE_LONG;
    // a cached workspace of this shape (most recently used first)
    auto it = ctx->wss.begin();
    for (; it != ctx->wss.end(); ++it)
        if (it->built && it->ragged == (lens != nullptr) &&
            (lens ? it->lens == *lens : (it->B == B && it->T == T && it->fused == fused && it->lz == lz)))
            break;
    static const bool dbg_ws = getenv("AVC_DEBUG_WS") && getenv("AVC_DEBUG_WS")[0] == '1';
    if (dbg_ws)
        fprintf(stderr, "AVC_DEBUG_WS ensure_ws B=%d T=%d fused=%d lz=%d ragged=%d n=%d: %s (%zu cached)\n", B, T,
                (int)fused, (int)lz, (int)(lens != nullptr), n_iters, it != ctx->wss.end() ? "hit" : "new", ctx->wss.size());
    if (it != ctx->wss.end()) {
        ctx->wss.splice(ctx->wss.begin(), ctx->wss, it);
        ctx->cur = &ctx->wss.front();
        if (n_iters <= ctx->cur->iters_cap) {
            ++ctx->n_ws_hits;
            return 0;
        }
    } else {
        // a new shape: make room (the stream may still use an evicted workspace's buffers)
        const char* ce = getenv("AVC_WS_CACHE");
        const int cap = std::max(1, ce ? atoi(ce) : ctx->ws_cap);
        while ((int)ctx->wss.size() >= cap) {
            HIPCHK(hipStreamSynchronize(ctx->stream));
            if (dbg_ws)
                fprintf(stderr, "AVC_DEBUG_WS evict ws B=%d T=%d lz=%d gen=%d\n", ctx->wss.back().B, ctx->wss.back().T,
                        (int)ctx->wss.back().lz, ctx->wss.back().gen);
            free_ws(ctx->wss.back());
            ctx->wss.pop_back();
            ++ctx->n_ws_evictions;
        }
        ctx->wss.emplace_front();
        ctx->cur = &ctx->wss.front();
    }
    Workspace& ws = *ctx->cur;
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (!ws.built) {
        ++ctx->n_ws_builds;
        ws.B = B;
        ws.T = T;
        ws.Tl = Tl;
        ws.X = X;
        ws.flop_fwd = flop;
        const int nb = ctx->nb;
        ws.fused = fused;
        ws.lz = lz;
        if (lens) {
            ws.ragged = true;
            ws.lens = *lens;
            std::vector<RagUtt> ru(B);
            int64_t off = 0;
            for (int b = 0; b < B; ++b) {
                ru[b] = RagUtt{};
                ru[b].T = (*lens)[b];
                ru[b].xoff = off;
                off += (int64_t)c.c_in * (*lens)[b];
            }
            WSCHK(hipMalloc(&ws.rag, B * sizeof(RagUtt)));
            WSCHK(hipMemcpy(ws.rag, ru.data(), B * sizeof(RagUtt), hipMemcpyHostToDevice));
        }
        int rc = 0;
        for (DevBuf* b : {&ws.xin, &ws.adv, &ws.vc, &ws.ptb, &ws.m, &ws.v, &ws.grad0}) rc |= dalloc(*b, X);
        for (DevBuf* b : {&ws.emb_fwd, &ws.org, &ws.tgt}) rc |= dalloc(*b, (size_t)B * c.c_out);
        if (ws.fused) {
            ws.mask_words = (nb + 1 + 2 * c.n_conv_blocks) * FZ_MASK_WORDS_PER_LAYER;
            rc |= dalloc(ws.pooled, (size_t)B * FZ_C);
            rc |= dalloc(ws.gpooled, (size_t)B * FZ_C);
            rc |= dalloc(ws.loss_cur, (size_t)B);
            if (rc) return drop_ws(ctx);
            WSCHK(hipMalloc(&ws.masks, (size_t)B * ws.mask_words * sizeof(unsigned long long)));
            if (ws.lz && alloc_long(ws.lza, B, T, nb + 1 + 2 * c.n_conv_blocks)) return drop_ws(ctx);
        } else {
            rc |= dalloc(ws.gxd, X);
            rc |= dalloc(ws.bank, (size_t)B * nb * c.c_bank * T);
            rc |= dalloc(ws.gbank, (size_t)B * nb * c.c_bank * T);
            const size_t H = (size_t)B * c.c_h * T;
            for (DevBuf* b : {&ws.h0, &ws.g1, &ws.ghx, &ws.ghy, &ws.gmx, &ws.gmy}) rc |= dalloc(*b, H);
            ws.a1.resize(c.n_conv_blocks);
            ws.a2.resize(c.n_conv_blocks);
            ws.hb.resize(c.n_conv_blocks);
            for (int l = 0; l < c.n_conv_blocks; ++l) {
                rc |= dalloc(ws.a1[l], (size_t)B * c.c_h * Tl[l]);
                rc |= dalloc(ws.a2[l], (size_t)B * c.c_h * Tl[l + 1]);
                rc |= dalloc(ws.hb[l], (size_t)B * c.c_h * Tl[l + 1]);
            }
            rc |= dalloc(ws.slab, (size_t)KSPLIT_MAX * std::max(c.c_h, c.c_in) * B * T);
        }
        if (rc) return drop_ws(ctx);
        WSCHK(hipMalloc(&ws.step, sizeof(int)));
        if (dalloc(ws.scal, 8)) return drop_ws(ctx);
    } else {
        ++ctx->n_ws_replans;   // more iterations than this workspace's tables hold
    }
    const int cap = std::max(n_iters, std::max(ws.iters_cap, 1));
    if (dalloc(ws.losses, (size_t)cap * B)) return drop_ws(ctx);
    if (dalloc(ws.table, (size_t)cap * 2)) return drop_ws(ctx);
    ws.iters_cap = cap;
    // (re)build plans: pointers may have moved (the bf16 plan is rebuilt on demand)
    free_plans(ws);
    ws.built = false;
    ws.gen = ++ctx->gen_next;
    if (ws.fused) {
        if (plan_fused_forward(ctx, ws, ws.fwd, ws.xin.p, false, PREC_F32)) return drop_ws(ctx);
    } else {
        if (plan_forward(ctx, ws, ws.fwd, ws.xin.p, false, PREC_F32)) return drop_ws(ctx);
    }
    if (plan_iteration(ctx, ws, ws.iter, PREC_F32)) return drop_ws(ctx);
    // autotune with a valid Adam step (1) and eps/gscale (the kernels clamp anyway)
    const float scal0[8] = {0.1f, 0.f, 0.f, 0.f, 0.1f, 0.f, 0.f, 0.f};
    WSCHK(hipMemcpy(ws.scal.p, scal0, sizeof(scal0), hipMemcpyHostToDevice));
    WSCHK(hipMemset(ws.step, 0, sizeof(int)));
    if (autotune(ctx, ws.fwd) || autotune(ctx, ws.iter)) return drop_ws(ctx);
    ws.built = true;
    return 0;
}

// Kernel-timestamp events for profiled launches: hipExtLaunchKernelGGL stamps the
// dispatch packet itself (the same start/end rocprofv3 reports), so per-kernel
// averages carry no event-record overhead.  Null => plain launch (graph capture).
struct KEv {
    hipEvent_t gemm0 = nullptr, gemm1 = nullptr;   // conv_gemm
    hipEvent_t red0 = nullptr, red1 = nullptr;     // splitk_reduce (when ksplit > 1)
};

template <typename F, typename... Args>
static void klaunch(const KEv* ev, bool reduce, F kernel, dim3 g, dim3 blk, unsigned shmem, hipStream_t s,
                    Args... args) {
    if (ev)
        hipExtLaunchKernelGGL(kernel, g, blk, shmem, s, reduce ? ev->red0 : ev->gemm0,
                              reduce ? ev->red1 : ev->gemm1, 0, args...);
    else
        hipLaunchKernelGGL(kernel, g, blk, shmem, s, args...);
}

template <int PREC, int WM, int WN, int WGM, int WGN, int KC>
static void launch_variant(const Launch& L, dim3 g, hipStream_t s, const KEv* ev) {
    const dim3 blk(64 * WGM * WGN);
    const int st = (L.stride == 1 || L.stride == 2) ? L.stride : 0;
#define AVC_L(MODE, ST) \
    klaunch(ev, false, conv_gemm<PREC, WM, WN, WGM, WGN, KC, MODE, ST>, g, blk, 0, s, L.dprobs, L.ksplit)
    if (L.mode == SEG_FWD) {
        if (st == 1) AVC_L(SEG_FWD, 1);
        else if (st == 2) AVC_L(SEG_FWD, 2);
        else AVC_L(SEG_FWD, 0);
    } else {
        if (st == 1) AVC_L(SEG_BWD, 1);
        else if (st == 2) AVC_L(SEG_BWD, 2);
        else AVC_L(SEG_BWD, 0);
    }
#undef AVC_L
}

static hipError_t launch_gemm(const Launch& L, int variant, hipStream_t s, const KEv* ev = nullptr) {
    if (variant < 0 || variant >= NVARIANTS || !variant_fits(L, variant)) return hipErrorInvalidValue;
    const dim3 g = gemm_grid(L, variant);
    switch (variant) {
#define AVC_GEMM_VARIANT(I, PREC, WM, WN, WGM, WGN, KC, NAME) \
    case I:                                                   \
        launch_variant<PREC, WM, WN, WGM, WGN, KC>(L, g, s, ev); \
        break;
#include "avc_gemm_variants.h"
#undef AVC_GEMM_VARIANT
    default:
        return hipErrorInvalidValue;
    }
    if (L.ksplit > 1) {
        const long groups = (long)L.maxM * cdiv(L.maxN, 4);
        klaunch(ev, true, splitk_reduce, dim3((unsigned)cdiv((int)groups, 256), 1, L.nprob), dim3(256), 0, s,
                L.dprobs, L.ksplit);
    }
    return hipGetLastError();
}

static hipError_t launch_one(const Launch& L, hipStream_t s, const KEv* ev = nullptr) {
    switch (L.kind) {
    case L_GEMM:
        return launch_gemm(L, L.variant, s, ev);
    case L_HEAD:
        klaunch(ev, false, se_head, L.grid, L.block, L.shmem, s, L.head);
        return hipGetLastError();
    case L_HEAD_V:
        if (L.prec == PREC_BF16) klaunch(ev, false, se_head_v<true>, L.grid, L.block, L.shmem, s, L.head);
        else klaunch(ev, false, se_head_v<false>, L.grid, L.block, L.shmem, s, L.head);
        return hipGetLastError();
    case L_FZ_FWD:
    case L_FZ_BWD: {
        typedef void (*FzK)(FusedArgs);
#define AVC_FZ_K(SH)                                                                                  \
    (L.kind == L_FZ_FWD ? (L.prec == PREC_F32 ? (FzK)se_fwd_fused<PREC_F32, SH> : (FzK)se_fwd_fused<PREC_BF16, SH>) \
                        : (L.prec == PREC_F32 ? (FzK)se_bwd_fused<PREC_F32, SH> : (FzK)se_bwd_fused<PREC_BF16, SH>))
        const FzK k = L.fz_shape == 0 ? AVC_FZ_K(0)
                      : L.fz_shape == 1 ? AVC_FZ_K(1)
                      : L.fz_shape == 2 ? AVC_FZ_K(2)
                      : L.fz_shape == 4 ? AVC_FZ_K(4)
                      : L.fz_shape == 16 ? AVC_FZ_K(16)
                                        : AVC_FZ_K(8);
#undef AVC_FZ_K
        klaunch(ev, false, k, L.grid, L.block, L.shmem, s, L.fz);
        return hipGetLastError();
    }
    case L_DZ_FWD:
    case L_DZ_BWD: {
        typedef void (*DzK)(DecArgs);
#define AVC_DZ_K(SH)                                                                                   \
    (L.kind == L_DZ_FWD ? (L.prec == PREC_F32 ? (DzK)dec_fwd_fused<PREC_F32, SH> : (DzK)dec_fwd_fused<PREC_BF16, SH>) \
                        : (L.prec == PREC_F32 ? (DzK)dec_bwd_fused<PREC_F32, SH> : (DzK)dec_bwd_fused<PREC_BF16, SH>))
        const DzK k = L.fz_shape == 0 ? AVC_DZ_K(0) : AVC_DZ_K(8);
#undef AVC_DZ_K
        klaunch(ev, false, k, L.grid, L.block, L.shmem, s, L.dz);
        return hipGetLastError();
    }
    case L_DENSE:
        // fp32 MFMA tiles when the rows take 16-byte loads (K, kchunk multiples of 4; always on
        // the AdaIN-VC config), the VALU kernel otherwise
        if (L.dn.variant == DZ_LDS)
            klaunch(ev, false, dense_lds, L.grid, L.block, L.shmem, s, L.dn);
        else if (L.dn.variant == DZ_MFMA)
            klaunch(ev, false, dense_mfma<2>, L.grid, L.block, 0, s, L.dn);
        else
            klaunch(ev, false, dense_batched, L.grid, L.block, 0, s, L.dn);
        return hipGetLastError();
    case L_HDR_COMPOSE:
        klaunch(ev, false, hdr_compose, L.grid, L.block, 0, s, L.hd);
        return hipGetLastError();
    case L_SN_POWER:
        klaunch(ev, false, sn_power, L.grid, L.block, 0, s, L.sn);
        return hipGetLastError();
    case L_SN_SCALE:
        klaunch(ev, false, sn_scale, L.grid, L.block, 0, s, L.sn);
        return hipGetLastError();
    case L_HDR_UPDATE:
        klaunch(ev, false, hdr_update, L.grid, L.block, 0, s, L.hd);
        return hipGetLastError();
    case L_LZ_FWD:
        if (L.prec == PREC_F32) klaunch(ev, false, lz_se_fwd<PREC_F32>, L.grid, L.block, L.shmem, s, L.fz, L.lz);
        else klaunch(ev, false, lz_se_fwd<PREC_BF16>, L.grid, L.block, L.shmem, s, L.fz, L.lz);
        return hipGetLastError();
    case L_LZ_BWD:
        if (L.prec == PREC_F32) klaunch(ev, false, lz_se_bwd<PREC_F32>, L.grid, L.block, L.shmem, s, L.fz, L.lz);
        else klaunch(ev, false, lz_se_bwd<PREC_BF16>, L.grid, L.block, L.shmem, s, L.fz, L.lz);
        return hipGetLastError();
    case L_LZD_FWD:
        if (L.prec == PREC_F32) klaunch(ev, false, lz_dec_fwd<PREC_F32>, L.grid, L.block, L.shmem, s, L.dz, L.lz);
        else klaunch(ev, false, lz_dec_fwd<PREC_BF16>, L.grid, L.block, L.shmem, s, L.dz, L.lz);
        return hipGetLastError();
    case L_LZD_BWD:
        if (L.prec == PREC_F32) klaunch(ev, false, lz_dec_bwd<PREC_F32>, L.grid, L.block, L.shmem, s, L.dz, L.lz);
        else klaunch(ev, false, lz_dec_bwd<PREC_BF16>, L.grid, L.block, L.shmem, s, L.dz, L.lz);
        return hipGetLastError();
    default:
        return hipErrorInvalidValue;
    }
}

static std::string kernel_name(const Launch& L) {
    return L.kind == L_GEMM ? std::string(VARIANTS[L.variant].name) : L.name;
}

// Time every tile variant of every GEMM launch of `pl` on the ctx stream and keep
// the fastest (median of 5 after a warm-up).  Runs once per workspace build.
// Tune cache (AVC_TUNE_FILE): lines "key variant" so a profiled re-run (rocprofv3)
// replays the same tile choices without the tuning launches.
static std::string tune_key(avc_ctx* ctx, const Plan& pl, size_t li) {
    char buf[256];
    const avc_se_cfg& c = ctx->cfg;
    snprintf(buf, sizeof(buf), "B%d_T%d_ch%d_%d_%d_nb%d_%s_l%zu", ctx->cur->B, ctx->cur->T, c.c_in, c.c_h, c.c_bank,
             c.n_conv_blocks, &pl == &ctx->cur->fwd ? "fwd" : (&pl == &ctx->cur->iter ? "iter" : "iterbf16"), li);
    return buf;
}

static std::map<std::string, int> read_tune_file() {
    std::map<std::string, int> m;
    const char* path = getenv("AVC_TUNE_FILE");
    if (!path) return m;
    FILE* f = fopen(path, "r");
    if (!f) return m;
    char key[256];
    int v;
    while (fscanf(f, "%255s %d", key, &v) == 2) m[key] = v;
    fclose(f);
    return m;
}

// AVC_PRINT_PLAN=1: one stderr line per launch of a tuned plan (position, layer,
// kernel, grid, split-K) -- lets a rocprofv3 trace be read layer by layer.
static void print_plan(avc_ctx* ctx, const Plan& pl) {
    if (!getenv("AVC_PRINT_PLAN")) return;
    const char* tag = &pl == &ctx->cur->fwd ? "fwd" : (&pl == &ctx->cur->iter ? "iter" : "iterbf16");
    for (size_t i = 0; i < pl.launches.size(); ++i) {
        const Launch& L = pl.launches[i];
        const dim3 g = L.kind == L_GEMM ? gemm_grid(L, L.variant) : L.grid;
        fprintf(stderr, "plan %s %zu %s %s grid=%u,%u,%u ksplit=%d flop=%.4g\n", tag, i, L.name.c_str(),
                L.kind == L_GEMM ? VARIANTS[L.variant].name : L.name.c_str(), g.x, g.y, g.z,
                L.ksplit, L.flop);
    }
}

static int autotune_(avc_ctx* ctx, Plan& pl);
static int autotune(avc_ctx* ctx, Plan& pl) {
    const int rc = autotune_(ctx, pl);
    if (!rc) print_plan(ctx, pl);
    return rc;
}

static int autotune_(avc_ctx* ctx, Plan& pl) {
    const char* env = getenv("AVC_AUTOTUNE");
    if (env && env[0] == '0') return 0;
    std::map<std::string, int> cache = read_tune_file();
    bool all_cached = true;
    for (size_t li = 0; li < pl.launches.size(); ++li) {
        if (pl.launches[li].kind != L_GEMM) continue;
        auto it = cache.find(tune_key(ctx, pl, li));
        if (it == cache.end() || it->second < 0 || it->second >= NVARIANTS ||
            !variant_fits(pl.launches[li], it->second))
            all_cached = false;
    }
    if (all_cached) {
        for (size_t li = 0; li < pl.launches.size(); ++li)
            if (pl.launches[li].kind == L_GEMM) pl.launches[li].variant = cache[tune_key(ctx, pl, li)];
        return 0;
    }
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    for (Launch& L : pl.launches) {
        if (L.kind != L_GEMM) continue;
        int best = L.variant;
        float best_ms = 1e30f;
        for (int v = 0; v < NVARIANTS; ++v) {
            if (!variant_fits(L, v)) continue;
            float t[5];
            HIPCHK(launch_gemm(L, v, ctx->stream));
            for (int r = 0; r < 5; ++r) {
                HIPCHK(hipEventRecord(a, ctx->stream));
                HIPCHK(launch_gemm(L, v, ctx->stream));
                HIPCHK(hipEventRecord(b, ctx->stream));
                HIPCHK(hipEventSynchronize(b));
                HIPCHK(hipEventElapsedTime(&t[r], a, b));
            }
            std::sort(t, t + 5);
            if (t[2] < best_ms) {
                best_ms = t[2];
                best = v;
            }
        }
        L.variant = best;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (const char* path = getenv("AVC_TUNE_FILE")) {
        if (FILE* f = fopen(path, "a")) {
            for (size_t li = 0; li < pl.launches.size(); ++li)
                if (pl.launches[li].kind == L_GEMM)
                    fprintf(f, "%s %d\n", tune_key(ctx, pl, li).c_str(), pl.launches[li].variant);
            fclose(f);
        }
    }
    return 0;
}

static void prof_add(avc_ctx* ctx, const std::string& nm, float ms, double flop) {
    auto& s = ctx->prof[nm];
    s.first += ms;
    s.second += flop;
    ctx->prof_n[nm] += 1;
}

static int run_plan(avc_ctx* ctx, const Plan& pl, bool prof) {
    KEv ev;
    if (prof)
        for (hipEvent_t* e : {&ev.gemm0, &ev.gemm1, &ev.red0, &ev.red1}) HIPCHK(hipEventCreate(e));
    static const bool dbg_sync = getenv("AVC_DEBUG_SYNC") && getenv("AVC_DEBUG_SYNC")[0] == '1';
    for (const Launch& L : pl.launches) {
        hipError_t e = launch_one(L, ctx->stream, prof ? &ev : nullptr);
        if (e != hipSuccess) return fail("launch %s: %s", kernel_name(L).c_str(), hipGetErrorString(e));
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (dbg_sync) (void)hipStreamIsCapturing(ctx->stream, &cs);
        if (dbg_sync && cs == hipStreamCaptureStatusNone) {   // diagnostics: each launch completes before the next
            e = hipStreamSynchronize(ctx->stream);
            if (e != hipSuccess) {
                fprintf(stderr, "AVC_DEBUG_SYNC: %s failed: %s\n", kernel_name(L).c_str(), hipGetErrorString(e));
                return fail("kernel %s: %s", kernel_name(L).c_str(), hipGetErrorString(e));
            }
        }
        if (!prof) continue;
        const bool red = L.kind == L_GEMM && L.ksplit > 1;
        HIPCHK(hipEventSynchronize(red ? ev.red1 : ev.gemm1));
        float ms = 0, ms_red = 0;
        HIPCHK(hipEventElapsedTime(&ms, ev.gemm0, ev.gemm1));
        if (red) HIPCHK(hipEventElapsedTime(&ms_red, ev.red0, ev.red1));
        const std::string nm = kernel_name(L);
        prof_add(ctx, nm, ms, L.flop);
        if (red) prof_add(ctx, "splitk_reduce", ms_red, 0.0);
        if (getenv("AVC_PROFILE_ROLES"))   // per-layer breakdown (diagnostics), reduce included
            prof_add(ctx, "role:" + L.name + "|" + nm, ms + ms_red, L.flop);
    }
    if (prof)
        for (hipEvent_t e : {ev.gemm0, ev.gemm1, ev.red0, ev.red1}) (void)hipEventDestroy(e);
    return 0;
}

static int begin_call(avc_ctx* ctx, hipStream_t user) {
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipEventRecord(ctx->ev_user, user));
    HIPCHK(hipStreamWaitEvent(ctx->stream, ctx->ev_user, 0));
    return 0;
}

static int end_call(avc_ctx* ctx, hipStream_t user) {
    HIPCHK(hipEventRecord(ctx->ev_done, ctx->stream));
    HIPCHK(hipStreamWaitEvent(user, ctx->ev_done, 0));
    return 0;
}

extern "C" int avc_se_forward(avc_ctx* ctx, const float* x, int B, int T, float* emb, void* stream) {
    if (!ctx || !x || !emb) return fail("avc_se_forward: null argument");
    hipStream_t us = (hipStream_t)stream;
    if (ensure_ws(ctx, B, T, 1)) return 1;
    if (begin_call(ctx, us)) return 1;
    Workspace& ws = *ctx->cur;
    const avc_se_cfg& c = ctx->cfg;
    HIPCHK(hipMemcpyAsync(ws.xin.p, x, (size_t)B * c.c_in * T * sizeof(float), hipMemcpyDeviceToDevice,
                          ctx->stream));
    if (run_plan(ctx, ws.fwd, false)) return 1;
    HIPCHK(hipMemcpyAsync(emb, ws.emb_fwd.p, (size_t)B * c.c_out * sizeof(float), hipMemcpyDeviceToDevice,
                          ctx->stream));
    return end_call(ctx, us);
}

extern "C" int avc_set_engine(avc_ctx* ctx, int engine) {
    if (!ctx) return fail("null ctx");
    if (engine != AVC_ENGINE_AUTO && engine != AVC_ENGINE_LAYERED && engine != AVC_ENGINE_FUSED &&
        engine != AVC_ENGINE_LONG)
        return fail("bad engine %d", engine);
    if ((engine == AVC_ENGINE_FUSED || engine == AVC_ENGINE_LONG) && !ctx->fused_ok)
        return fail("the fused engine needs c_in=80, c_h=c_bank=c_out=128, bank_scale=1, bank_size<=8, odd kernel_size<=5, "
                    "<=8 conv blocks with subsample 1 or 2");
    ctx->engine = engine;
    return 0;
}

extern "C" int avc_get_engine(avc_ctx* ctx, int T) {
    if (!ctx) return -1;
    return engine_for(ctx, T);
}

// In-graph kernel timing (avc_ktime.h): the records of each kernel translation unit
extern "C" avc::KTime* avc_ktime_records_fused();
extern "C" avc::KTime* avc_ktime_records_long();
extern "C" avc::KTime* avc_ktime_records_vc();

extern "C" int avc_ktime(avc_ctx* ctx, int enable, double* avg_us, int64_t* launches) {
    if (!ctx) return fail("avc_ktime: null context");
    HIPCHK(hipSetDevice(ctx->device));
    // the records are per device, shared by every context and stream on it: drain the whole device, so no
    // stamped kernel of another context can race the read-out / reset below
    HIPCHK(hipDeviceSynchronize());
    avc::KTime* units[3] = {avc_ktime_records_fused(), avc_ktime_records_long(), avc_ktime_records_vc()};
    // output order: fused slots 0-3, long 0-7, Decoder 0-3, then fused 4-5 (se_attack_fused)
    const int used[3] = {4, 8, 4};   // records in use per unit (avc_ktime.h slots) before the appended ones
    int rate_khz = 0;
    HIPCHK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, ctx->device));
    int o = 0;
    for (int u = 0; u < 3; ++u) {
        if (!units[u]) return fail("avc_ktime: kernel timing records not found");
        avc::KTime h[avc::KT_SLOTS];
        HIPCHK(hipMemcpy(h, units[u], sizeof(h), hipMemcpyDeviceToHost));
        auto put = [&](int i, int at) {
            if (enable) return;
            if (avg_us) avg_us[at] = h[i].n && rate_khz > 0 ? (double)h[i].sum / (double)h[i].n / rate_khz * 1e3 : 0.0;
            if (launches) launches[at] = (int64_t)h[i].n;
        };
        for (int i = 0; i < used[u]; ++i, ++o) put(i, o);
        if (u == 0)
            for (int i = 0; i < 2; ++i) put(avc::KT_FUSED_ATK + i, 16 + i);
        for (int i = 0; i < avc::KT_SLOTS; ++i) {
            h[i] = avc::KTime{};
            h[i].on = enable ? 1ull : 0ull;
            h[i].t0 = ~0ull;
        }
        HIPCHK(hipMemcpy(units[u], h, sizeof(h), hipMemcpyHostToDevice));
    }
    return 0;
}

extern "C" int avc_set_profiling(avc_ctx* ctx, int enable) {
    if (!ctx) return fail("null ctx");
    ctx->profiling = enable != 0;
    ctx->prof.clear();
    ctx->prof_n.clear();
    ctx->prof_iters = 0;
    return 0;
}

// Adam scalars per step (computed in double like torch's Python-side math) and the per-call
// scalars [eps, loss-grad scales...] -> ws.table / ws.scal on ctx->stream, asynchronously
// through the pinned staging buffer
static int stage_call_consts(avc_ctx* ctx, int n_iters, const float scal[4], double lr = 1e-3, double beta1 = 0.9,
                             double beta2 = 0.999, float lam = 0.1f, int t0 = 0) {
    Workspace& ws = *ctx->cur;
    const size_t nt = 2 * (size_t)std::max(n_iters, 1);
    HIPCHK(hipEventSynchronize(ctx->ev_stage));   // the previous call's staging copies are done
    if (ctx->stage_n < nt + 8) {
        if (ctx->stage) (void)hipHostFree(ctx->stage);
        ctx->stage = nullptr;
        ctx->stage_n = 0;
        HIPCHK(hipHostMalloc((void**)&ctx->stage, (nt + 8) * sizeof(float), hipHostMallocDefault));
        ctx->stage_n = nt + 8;
    }
    float* table = ctx->stage;
    for (size_t i = 0; i < nt; ++i) table[i] = 0.f;
    for (int t = 1; t <= n_iters; ++t) {   // step t0 + t of the optimiser (t0 steps taken before this call)
        const double bc1 = 1.0 - std::pow(beta1, t0 + t);
        const double bc2 = 1.0 - std::pow(beta2, t0 + t);
        table[2 * (t - 1)] = (float)(-(lr / bc1));
        table[2 * (t - 1) + 1] = (float)std::sqrt(bc2);
    }
    for (int i = 0; i < 4; ++i) table[nt + i] = scal[i];
    table[nt + 4] = lam;
    for (int i = 5; i < 8; ++i) table[nt + i] = 0.f;
    HIPCHK(hipMemcpyAsync(ws.table.p, table, nt * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ws.scal.p, table + nt, 8 * sizeof(float), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipEventRecord(ctx->ev_stage, ctx->stream));
    return 0;
}

// Graph replay of an iteration plan: GRAPH_ITERS iterations are captured into ONE graph (the Adam step
// counter lives in HBM, so consecutive iterations are identical launches) -- a graph launch
// per iteration left ~9 us between the backward's end and the next forward's start (kernel
// trace), against none between the kernels inside a graph.  The n_iters % GRAPH_ITERS tail runs as
// plain launches.
// The persistent emb attack (se_attack_fused): a bf16 emb iteration plan of the fused forward with the head
// in its tail and the fused backward + Adam, at the standard shape (T = 128), runs all its iterations in ONE launch
// (then fz_step_add advances the step counter by as many).  AVC_PERSIST=0 keeps the per-pass launches.
static bool persist_ok(const Plan& iter) {
    const char* e = getenv("AVC_PERSIST");   // (read per call: tests compare both paths in one process)
    const bool off = e && e[0] == '0';
    const char* e16 = getenv("AVC_PERSIST16");   // A/B: the runtime-length shape on per-pass launches
    const bool persist16_off = e16 && e16[0] == '0';
    if (off || iter.launches.size() != 2) return false;
    const Launch& F = iter.launches[0];
    const Launch& Bk = iter.launches[1];
    return F.kind == L_FZ_FWD && Bk.kind == L_FZ_BWD && F.prec == PREC_BF16 && Bk.prec == PREC_BF16 &&
           F.fz.fuse_head == 1 && F.fz_shape == Bk.fz_shape && (F.fz_shape == 0 || (F.fz_shape == 16 && !persist16_off)) &&
           !Bk.fz.gx_out && Bk.fz.fuse_head == 0 && F.fz.tick == Bk.fz.step && !F.fz.rag;
}
static int run_persist(avc_ctx* ctx, const Plan& iter, int n_iters) {
    if (n_iters <= 0) return 0;
    const Launch& F = iter.launches[0];
    const Launch& Bk = iter.launches[1];
    AtkArgs a;
    a.f = F.fz;
    a.f.tick = nullptr;   // the counter moves once per launch (fz_step_add), not per forward
    a.b = Bk.fz;
    a.n_iters = n_iters;
    const size_t sh = std::max(F.shmem, Bk.shmem);
    if (F.fz_shape == 0) hipLaunchKernelGGL((se_attack_fused<PREC_BF16, 0>), F.grid, F.block, sh, ctx->stream, a);
    else hipLaunchKernelGGL((se_attack_fused<PREC_BF16, 16>), F.grid, F.block, sh, ctx->stream, a);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(fz_step_add, dim3(1), dim3(64), 0, ctx->stream, F.fz.tick, n_iters);
    HIPCHK(hipGetLastError());
    return 0;
}

constexpr int GRAPH_ITERS = 50;
static int graph_replay(avc_ctx* ctx, Plan& iter, hipGraphExec_t& graph, int n_iters) {
    const int nfull = n_iters / GRAPH_ITERS;
    if (nfull > 0 && !graph) {
        hipGraph_t g;
        HIPCHK(hipStreamBeginCapture(ctx->stream, hipStreamCaptureModeThreadLocal));
        int rc = 0;
        for (int it = 0; it < GRAPH_ITERS && !rc; ++it) rc = run_plan(ctx, iter, false);
        hipError_t e = hipStreamEndCapture(ctx->stream, &g);
        if (e == hipSuccess && rc) (void)hipGraphDestroy(g);
        if (rc) return 1;
        if (e != hipSuccess) return fail("graph capture: %s", hipGetErrorString(e));
        ++ctx->n_graph_captures;
        e = hipGraphInstantiate(&graph, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (e != hipSuccess) {
            graph = nullptr;
            return fail("graph instantiate: %s", hipGetErrorString(e));
        }
    }
    for (int it = 0; it < nfull; ++it) HIPCHK(hipGraphLaunch(graph, ctx->stream));
    for (int it = nfull * GRAPH_ITERS; it < n_iters; ++it)
        if (run_plan(ctx, iter, false)) return 1;
    return 0;
}

// emb attack; the target embedding is SE(adv_tgt) at T frames (adv_tgt given) or the caller's
// tgt_emb [B][c_out] (adv_tgt of another length, embedded beforehand by avc_se_forward)
static int emb_attack_impl(avc_ctx* ctx, const float* vc_tgt, const float* adv_tgt, const float* tgt_emb,
                           const float* ptb0, int B, int T, float eps, int n_iters, float* out_adv,
                           const avc_attack_opts* opts, void* stream, const std::vector<int>* lens = nullptr) {
    if (!ctx || !vc_tgt || !(adv_tgt || tgt_emb) || !ptb0 || !out_adv) return fail("avc_emb_attack: null argument");
    if (n_iters < 0) return fail("n_iters must be >= 0");
    avc_attack_opts o{};
    o.use_graph = 1;
    if (opts) o = *opts;
    if (o.precision != AVC_PREC_FP32 && o.precision != AVC_PREC_BF16) return fail("bad precision %d", o.precision);
    if (o.reduction != AVC_REDUCE_INDEPENDENT && o.reduction != AVC_REDUCE_MEAN)
        return fail("bad reduction %d", o.reduction);
    if (o.update != AVC_UPDATE_ADAM && !(o.update == AVC_UPDATE_PGD && o.pgd_step > 0.f))
        return fail("bad update %d (PGD needs pgd_step > 0)", o.update);
    hipStream_t us = (hipStream_t)stream;
    if (ensure_ws(ctx, B, T, n_iters, lens)) return 1;
    Workspace& ws = *ctx->cur;
    const bool bf16 = o.precision == AVC_PREC_BF16;
    if (bf16 && ws.iter_bf16.launches.empty()) {
        // the setup below rewrites eps and the step counter with blocking copies on the null
        // stream: an earlier (asynchronous) call's loop on ctx->stream must be finished first
        HIPCHK(hipStreamSynchronize(ctx->stream));
        if (plan_iteration(ctx, ws, ws.iter_bf16, PREC_BF16)) return 1;
        const float scal0[8] = {0.1f, 0.f, 0.f, 0.f, 0.1f, 0.f, 0.f, 0.f};
        HIPCHK(hipMemcpy(ws.scal.p, scal0, sizeof(scal0), hipMemcpyHostToDevice));
        HIPCHK(hipMemset(ws.step, 0, sizeof(int)));
        if (autotune(ctx, ws.iter_bf16)) return 1;
    }
    Plan& iter = bf16 ? ws.iter_bf16 : ws.iter;
    hipGraphExec_t& graph = bf16 ? ws.graph_bf16 : ws.graph;
    if (begin_call(ctx, us)) return 1;
    const avc_se_cfg& c = ctx->cfg;
    const size_t X = ws.X;   // B x 80 x T, or a ragged batch's packed sum
    const float gscale = (float)(2.0 / (o.reduction == AVC_REDUCE_MEAN ? (double)B * c.c_out : (double)c.c_out));

    const float scal[4] = {eps, gscale, 0.f, o.update == AVC_UPDATE_PGD ? o.pgd_step : 0.f};
    if (stage_call_consts(ctx, n_iters, scal)) return 1;
    HIPCHK(hipMemcpyAsync(ws.vc.p, vc_tgt, X * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    // org_emb = SE(vc_tgt), tgt_emb = SE(adv_tgt)   (attack_utils.py:73-75)
    HIPCHK(hipMemcpyAsync(ws.xin.p, vc_tgt, X * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    if (run_plan(ctx, ws.fwd, false)) return 1;
    HIPCHK(hipMemcpyAsync(ws.org.p, ws.emb_fwd.p, (size_t)B * c.c_out * sizeof(float), hipMemcpyDeviceToDevice,
                          ctx->stream));
    if (adv_tgt) {
        HIPCHK(hipMemcpyAsync(ws.xin.p, adv_tgt, X * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
        if (run_plan(ctx, ws.fwd, false)) return 1;
    }
    HIPCHK(hipMemcpyAsync(ws.tgt.p, adv_tgt ? ws.emb_fwd.p : tgt_emb, (size_t)B * c.c_out * sizeof(float),
                          hipMemcpyDeviceToDevice, ctx->stream));
    // ptb <- ptb0, Adam state 0, adv = vc + eps*tanh(ptb)
    hipLaunchKernelGGL(attack_init, dim3((unsigned)((X + 255) / 256)), dim3(256), 0, ctx->stream, ws.vc.p, ptb0,
                       ws.ptb.p, ws.m.p, ws.v.p, ws.adv.p, eps, X, o.update == AVC_UPDATE_PGD ? 1 : 0);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemsetAsync(ws.step, 0, sizeof(int), ctx->stream));

    if (ctx->profiling) {
        hipEvent_t a, b;
        HIPCHK(hipEventCreate(&a));
        HIPCHK(hipEventCreate(&b));
        HIPCHK(hipEventRecord(a, ctx->stream));
        for (int it = 0; it < n_iters; ++it)
            if (run_plan(ctx, iter, true)) return 1;
        HIPCHK(hipEventRecord(b, ctx->stream));
        HIPCHK(hipEventSynchronize(b));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, a, b));
        ctx->prof_iter_ms += ms;
        ctx->prof_iters += n_iters;
        hipEventDestroy(a);
        hipEventDestroy(b);
    } else if (persist_ok(iter)) {
        if (run_persist(ctx, iter, n_iters)) return 1;
    } else if (o.use_graph && n_iters > 0 && !(getenv("AVC_NO_GRAPH") && getenv("AVC_NO_GRAPH")[0] == '1')) {
        if (graph_replay(ctx, iter, graph, n_iters)) return 1;
    } else {
        for (int it = 0; it < n_iters; ++it)
            if (run_plan(ctx, iter, false)) return 1;
    }
    HIPCHK(hipMemcpyAsync(out_adv, ws.adv.p, X * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    if (o.losses && n_iters > 0)
        HIPCHK(hipMemcpyAsync(o.losses, ws.losses.p, (size_t)n_iters * B * sizeof(float), hipMemcpyDeviceToDevice,
                              ctx->stream));
    if (o.grad0 && n_iters > 0)
        HIPCHK(hipMemcpyAsync(o.grad0, ws.grad0.p, X * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    return end_call(ctx, us);
}

extern "C" int avc_emb_attack(avc_ctx* ctx, const float* vc_tgt, const float* adv_tgt, const float* ptb0, int B,
                              int T, float eps, int n_iters, float* out_adv, const avc_attack_opts* opts,
                              void* stream) {
    if (!adv_tgt) return fail("avc_emb_attack: null argument");
    return emb_attack_impl(ctx, vc_tgt, adv_tgt, nullptr, ptb0, B, T, eps, n_iters, out_adv, opts, stream);
}

extern "C" int avc_emb_attack_emb(avc_ctx* ctx, const float* vc_tgt, const float* tgt_emb, const float* ptb0, int B,
                                  int T, float eps, int n_iters, float* out_adv, const avc_attack_opts* opts,
                                  void* stream) {
    if (!tgt_emb) return fail("avc_emb_attack_emb: null argument");
    return emb_attack_impl(ctx, vc_tgt, nullptr, tgt_emb, ptb0, B, T, eps, n_iters, out_adv, opts, stream);
}

// A ragged batch: utterance b has lengths[b] frames (host array); vc_tgt / ptb0 / out_adv (and opts->grad0)
// are packed [80][lengths[b]] blocks in batch order, tgt_emb [B][c_out] = SE(adv_tgt_b) at adv_tgt_b's own
// length.  One launch per pass over every length (the long engine with per-workgroup lengths).
extern "C" int avc_emb_attack_ragged(avc_ctx* ctx, const float* vc_tgt, const int* lengths, int B, const float* tgt_emb,
                                     const float* ptb0, float eps, int n_iters, float* out_adv,
                                     const avc_attack_opts* opts, void* stream) {
    if (!ctx || !lengths || !tgt_emb) return fail("avc_emb_attack_ragged: null argument");
    if (B <= 0) return fail("avc_emb_attack_ragged: batch size must be positive (got %d)", B);
    if (opts && opts->reduction != AVC_REDUCE_INDEPENDENT)
        return fail("avc_emb_attack_ragged: only independent per-utterance attacks (reduction 0)");
    const std::vector<int> lens(lengths, lengths + B);
    return emb_attack_impl(ctx, vc_tgt, nullptr, tgt_emb, ptb0, B, 0, eps, n_iters, out_adv, opts, stream, &lens);
}

static int run_iterations(avc_ctx* ctx, Plan& iter, hipGraphExec_t& graph, int n_iters, bool use_graph);

// UniversalPerturbationHeader.optimize (models/header_model.py:25-68) driven as
// train_header.py:46,77-80 does (torch Adam on the header): per iteration one captured graph
// of  hdr_compose -> SpeakerEncoder forward (+ loss, head backward) -> input-gradient pass
// (gx_out) -> hdr_update.  MSE means over all N x c_out elements (F.mse_loss on the batch).
static int plan_header(avc_ctx* ctx, Workspace& ws, Plan& pl, int prec, int N, int FT) {
    Launch C;
    C.kind = L_HDR_COMPOSE;
    C.grid = dim3((unsigned)std::min<size_t>(((size_t)N * FT + 255) / 256, 8192));
    C.block = dim3(256);
    C.name = "hdr_compose";
    HdrArgs& H = C.hd;
    H.src = ws.vc.p;
    H.hdr = ws.hdr.p;
    H.m = ws.hdr_m.p;
    H.v = ws.hdr_v.p;
    H.x = ws.adv.p;
    H.gx = ws.hdr_gx.p;
    H.table = ws.table.p;
    H.step = ws.step;
    H.table_len = ws.iters_cap;
    H.N = N;
    H.FT = FT;
    pl.launches.push_back(C);
    if (plan_fused_forward(ctx, ws, pl, ws.adv.p, true, prec) || plan_fused_backward(ctx, ws, pl, prec)) return 1;
    Launch& Bk = pl.launches.back();
    Bk.fz.gx_out = ws.hdr_gx.p;
    const Launch& F = pl.launches[pl.launches.size() - 2];
    if ((F.kind == L_FZ_FWD) && F.fz.fuse_head) {   // the fused head's loss row, written by the bwd
        Bk.fz.loss_cur = ws.loss_cur.p;
        Bk.fz.losses = ws.losses.p;
        Bk.fz.loss_len = ws.iters_cap;
    }
    Launch U = C;
    U.kind = L_HDR_UPDATE;
    U.grid = dim3((unsigned)((FT + 255) / 256));
    U.name = "hdr_update";
    pl.launches.push_back(U);
    return 0;
}

static int header_optimize_impl(avc_ctx* ctx, const float* source, const float* target, int N, int T, float* header,
                                float epsilon, float lambda_param, float lr, float beta1, float beta2, float adam_eps,
                                int n_iters, int precision, float* losses, float* exp_avg, float* exp_avg_sq,
                                int step0, void* stream) {
    if (!ctx || !source || !target || !header) return fail("avc_header_optimize: null argument");
    if (n_iters < 0) return fail("n_iters must be >= 0");
    if (step0 < 0) return fail("avc_header_optimize_state: step0 must be >= 0");
    if ((exp_avg == nullptr) != (exp_avg_sq == nullptr))
        return fail("avc_header_optimize_state: give both exp_avg and exp_avg_sq, or neither");
    if (step0 > 0 && !exp_avg) return fail("avc_header_optimize_state: step0 > 0 needs the Adam moments");
    if (precision != AVC_PREC_FP32 && precision != AVC_PREC_BF16) return fail("bad precision %d", precision);
    if (!(lr > 0.f) || !(beta1 >= 0.f && beta1 < 1.f) || !(beta2 >= 0.f && beta2 < 1.f) || !(adam_eps >= 0.f))
        return fail("avc_header_optimize: bad Adam hyper-parameters");
    hipStream_t us = (hipStream_t)stream;
    if (ensure_ws(ctx, N, T, n_iters)) return 1;
    Workspace& ws = *ctx->cur;
    if (!ws.fused) return fail("the header optimiser runs on the fused / long engine (not LAYERED)");
    const avc_se_cfg& c = ctx->cfg;
    const int FT = c.c_in * T;
    const size_t X = (size_t)N * FT;
    int rc = dalloc(ws.hdr, FT) | dalloc(ws.hdr_m, FT) | dalloc(ws.hdr_v, FT) | dalloc(ws.hdr_gx, X);
    if (rc) return 1;
    const int p = precision == AVC_PREC_BF16 ? 1 : 0;
    Plan& pl = ws.hdr_it[p];
    if (pl.launches.empty()) {
        HIPCHK(hipStreamSynchronize(ctx->stream));
        if (plan_header(ctx, ws, pl, p ? PREC_BF16 : PREC_F32, N, FT)) return 1;
    }
    for (Launch& L : pl.launches)
        if (L.kind == L_HDR_COMPOSE || L.kind == L_HDR_UPDATE) {
            L.hd.b1c = (float)(1.0 - (double)beta1);
            L.hd.b2 = beta2;
            L.hd.b2c = (float)(1.0 - (double)beta2);
            L.hd.adam_eps = adam_eps;
            L.hd.clamp_eps = epsilon;
        }
    hipGraphExec_t& graph = ws.hdr_graph[p];
    if (graph) {   // the Adam / clamp constants live in the kernel arguments: re-capture
        (void)hipGraphExecDestroy(graph);
        graph = nullptr;
    }
    if (begin_call(ctx, us)) return 1;
    const float gscale = (float)(2.0 / ((double)N * c.c_out));
    const float scal[4] = {epsilon, gscale, 0.f, 0.f};
    if (stage_call_consts(ctx, n_iters, scal, lr, beta1, beta2, lambda_param, step0)) return 1;
    // source_embedding = SE(source), target_embedding = SE(target)   (header_model.py:48-49)
    HIPCHK(hipMemcpyAsync(ws.vc.p, source, X * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ws.xin.p, source, X * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    if (run_plan(ctx, ws.fwd, false)) return 1;
    HIPCHK(hipMemcpyAsync(ws.org.p, ws.emb_fwd.p, (size_t)N * c.c_out * sizeof(float), hipMemcpyDeviceToDevice,
                          ctx->stream));
    HIPCHK(hipMemcpyAsync(ws.xin.p, target, X * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    if (run_plan(ctx, ws.fwd, false)) return 1;
    HIPCHK(hipMemcpyAsync(ws.tgt.p, ws.emb_fwd.p, (size_t)N * c.c_out * sizeof(float), hipMemcpyDeviceToDevice,
                          ctx->stream));
    HIPCHK(hipMemcpyAsync(ws.hdr.p, header, FT * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    if (exp_avg) {   // the caller's optimiser state (torch Adam exp_avg / exp_avg_sq)
        HIPCHK(hipMemcpyAsync(ws.hdr_m.p, exp_avg, FT * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(ws.hdr_v.p, exp_avg_sq, FT * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    } else {
        HIPCHK(hipMemsetAsync(ws.hdr_m.p, 0, FT * sizeof(float), ctx->stream));
        HIPCHK(hipMemsetAsync(ws.hdr_v.p, 0, FT * sizeof(float), ctx->stream));
    }
    HIPCHK(hipMemsetAsync(ws.step, 0, sizeof(int), ctx->stream));
    if (run_iterations(ctx, pl, graph, n_iters, true)) return 1;
    HIPCHK(hipMemcpyAsync(header, ws.hdr.p, FT * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    if (exp_avg) {
        HIPCHK(hipMemcpyAsync(exp_avg, ws.hdr_m.p, FT * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
        HIPCHK(hipMemcpyAsync(exp_avg_sq, ws.hdr_v.p, FT * sizeof(float), hipMemcpyDeviceToDevice, ctx->stream));
    }
    if (losses && n_iters > 0)
        HIPCHK(hipMemcpyAsync(losses, ws.losses.p, (size_t)n_iters * N * sizeof(float), hipMemcpyDeviceToDevice,
                              ctx->stream));
    return end_call(ctx, us);
}

extern "C" int avc_header_optimize(avc_ctx* ctx, const float* source, const float* target, int N, int T,
                                   float* header, float epsilon, float lambda_param, float lr, float beta1,
                                   float beta2, float adam_eps, int n_iters, int precision, float* losses,
                                   void* stream) {
    return header_optimize_impl(ctx, source, target, N, T, header, epsilon, lambda_param, lr, beta1, beta2, adam_eps,
                                n_iters, precision, losses, nullptr, nullptr, 0, stream);
}

extern "C" int avc_header_optimize_state(avc_ctx* ctx, const float* source, const float* target, int N, int T,
                                         float* header, float epsilon, float lambda_param, float lr, float beta1,
                                         float beta2, float adam_eps, int n_iters, int precision, float* losses,
                                         float* exp_avg, float* exp_avg_sq, int step0, void* stream) {
    return header_optimize_impl(ctx, source, target, N, T, header, epsilon, lambda_param, lr, beta1, beta2, adam_eps,
                                n_iters, precision, losses, exp_avg, exp_avg_sq, step0, stream);
}

extern "C" int avc_get_profile(avc_ctx* ctx, double* ms_per_iter, double* gemm_flop_per_iter) {
    if (!ctx) return fail("null ctx");
    if (ctx->prof_iters == 0) return fail("no profiled iterations");
    if (ms_per_iter) *ms_per_iter = ctx->prof_iter_ms / ctx->prof_iters;
    double f = 0;
    for (auto& kv : ctx->prof)
        if (kv.first.rfind("role:", 0) != 0) f += kv.second.second;
    if (gemm_flop_per_iter) *gemm_flop_per_iter = f / ctx->prof_iters;
    return 0;
}

extern "C" int avc_ws_stats(avc_ctx* ctx, int64_t* builds, int64_t* replans, int64_t* hits, int64_t* captures,
                            int64_t* evictions) {
    if (!ctx) return fail("null ctx");
    if (builds) *builds = ctx->n_ws_builds;
    if (replans) *replans = ctx->n_ws_replans;
    if (hits) *hits = ctx->n_ws_hits;
    if (captures) *captures = ctx->n_graph_captures;
    if (evictions) *evictions = ctx->n_ws_evictions;
    return 0;
}

extern "C" int avc_set_ws_cache(avc_ctx* ctx, int n_shapes) {
    if (!ctx) return fail("null ctx");
    if (n_shapes < 1 || n_shapes > 64) return fail("avc_set_ws_cache: n_shapes must be in [1, 64] (got %d)", n_shapes);
    ctx->ws_cap = n_shapes;
    return 0;
}

extern "C" int avc_profile_kernel_count(avc_ctx* ctx) { return ctx ? (int)ctx->prof.size() : 0; }

extern "C" int avc_profile_kernel(avc_ctx* ctx, int i, char* name, int name_len, long* launches, double* total_ms,
                                  double* total_flop) {
    if (!ctx || i < 0 || i >= (int)ctx->prof.size()) return fail("bad profile index");
    auto it = ctx->prof.begin();
    std::advance(it, i);
    if (name && name_len > 0) {
        strncpy(name, it->first.c_str(), name_len - 1);
        name[name_len - 1] = 0;
    }
    if (launches) *launches = ctx->prof_n[it->first];
    if (total_ms) *total_ms = it->second.first;
    if (total_flop) *total_flop = it->second.second;
    return 0;
}

#include "avc_vc_host.inc"
#include "avc_pm_host.inc"
#include "avc_dsp_host.inc"
