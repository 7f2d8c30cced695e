// fmha_api.cpp — the C ABI of libpaged-attention.so (declared in include/paged_attn.h).
//
// Re-implements the reference's L3 boundary (csrc/paged_attn.cpp:6-568): parameter packing
// (set_params_fprop_strided :6-126), the split heuristic (:128-163), split scratch (:165-196)
// and the three entry points (:310-568) — plus fmha_bwd / varlen / _ex entries the reference
// lacks.  Differences by design:
//   * no exceptions or exit() cross the ABI: failures set a thread-local error and return;
//   * split scratch comes from a cached per-(device, stream) pool — no hipMalloc/hipFree per call
//     (the reference mallocs every call and leaks, paged_attn.cpp:186-189,557-561);
//   * the current device is used (the reference queries device 0, :527-528);
//   * LSE is written whenever a pointer is given.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/paged_attn.h"
#include "fmha_launch.h"

using namespace xfa;

namespace xfa {
Options& options() {
    static Options o;
    return o;
}
thread_local char g_last_kernel[160] = "";   // kernel + schedule of this thread's last forward
void note_launch(const char* kernel, int persistent, int xcdq, unsigned gx, unsigned gy, unsigned gz, int block) {
    snprintf(g_last_kernel, sizeof(g_last_kernel), "%s persistent=%d xcdq=%d grid=%ux%ux%u block=%d",
             kernel, persistent, xcdq, gx, gy, gz, block);
}
}  // namespace xfa

namespace {

thread_local std::string g_err;
thread_local int g_status = 0;
thread_local int g_last_splits = 0;     // split count of this thread's last forward launch

void clear_error() { g_err.clear(); g_status = 0; }
// forward entries: also forget the last forward's kernel / splits, so a call that fails
// validation or launches nothing reports "" / 0 (fmha_last_kernel's contract)
void begin_fwd() { clear_error(); g_last_kernel[0] = 0; g_last_splits = 0; }
bool fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
bool fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    g_status = code;
    return false;
}
#define REQUIRE(cond, ...) do { if (!(cond)) { fail(1, __VA_ARGS__); return; } } while (0)

bool hip_ok(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    return fail(2, "%s: %s", what, hipGetErrorString(e));
}

// ---------------------------------------------------------------- scratch pool ---------
// One growable device buffer per (device, stream).  Work on a stream is ordered, so reuse
// by the next call on the same stream is safe; growth frees the old block (hipFree waits).
struct PoolEntry { void* ptr = nullptr; size_t bytes = 0; };
std::mutex g_pool_mu;
std::map<std::pair<int, hipStream_t>, PoolEntry> g_pool;

void* pool_get(hipStream_t st, size_t bytes) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    PoolEntry& e = g_pool[{dev, st}];
    if (e.bytes >= bytes) return e.ptr;
    if (e.ptr) { hipStreamSynchronize(st); hipFree(e.ptr); e.ptr = nullptr; e.bytes = 0; }
    size_t want = bytes + (bytes >> 3) + 4096;
    if (hipMalloc(&e.ptr, want) != hipSuccess) { e.ptr = nullptr; return nullptr; }
    e.bytes = want;
    return e.ptr;
}

// Item counters of the dynamic persistent forward (one pair of ints per (device, stream),
// zeroed once; the kernel's last workgroup resets them, so stream order keeps them valid).
std::map<std::pair<int, hipStream_t>, int*> g_ctr;
int* counter_get(hipStream_t st) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    int*& c = g_ctr[{dev, st}];
    if (!c) {
        if (hipMalloc(&c, 256) != hipSuccess) { c = nullptr; return nullptr; }
        if (hipMemsetAsync(c, 0, 256, st) != hipSuccess) { (void)hipFree(c); c = nullptr; return nullptr; }
    }
    return c;
}

// Split-arrival counters of the folded decode combine: >= n ints per (device, stream), zeroed
// when (re)allocated; every launch leaves them zero (the merging wave resets its counter).
std::map<std::pair<int, hipStream_t>, std::pair<int*, int>> g_dec_ctr;
int* dec_counters(hipStream_t st, int n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto& e = g_dec_ctr[{dev, st}];
    if (e.second >= n) return e.first;
    if (e.first) { hipStreamSynchronize(st); (void)hipFree(e.first); e.first = nullptr; e.second = 0; }
    const int want = std::max(n, 1024);
    if (hipMalloc(&e.first, (size_t)want * 4) != hipSuccess) { e.first = nullptr; return nullptr; }
    if (hipMemsetAsync(e.first, 0, (size_t)want * 4, st) != hipSuccess) { (void)hipFree(e.first); e.first = nullptr; return nullptr; }
    e.second = want;
    return e.first;
}

// CU count per device (a process may drive several GPUs; cached per device id)
int num_cus(int dev) {
    static std::mutex mu;
    static std::map<int, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(dev);
    if (it != cache.end()) return it->second;
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
    return n;
}
int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    return dev;
}

// Kernels address one sequence's rows of one tensor with 32-bit byte offsets from a buffer
// descriptor (and mark skipped lanes with kOOB = 0x7FFFFF00), so one sequence's slab of any
// tensor must stay below that (the reference's 64-bit index_t has no such limit; a slab this
// large is >= 256k tokens x 32 heads x d128 in bf16).
constexpr int64_t kMaxSlabBytes = 0x7FFFFF00LL;
bool slab_ok(const char* what, int64_t rows, int64_t row_elems, int esz) {
    const int64_t bytes = rows * row_elems * esz;
    if (bytes < kMaxSlabBytes) return true;
    return fail(1, "%s: one sequence spans %lld bytes (%lld rows x %lld elements); this build "
                "addresses a sequence with 32-bit offsets and supports < %lld bytes",
                what, (long long)bytes, (long long)rows, (long long)row_elems, (long long)kMaxSlabBytes);
}

// Reference heuristic (paged_attn.cpp:128-163): the smallest split count whose wave
// efficiency reaches 85% of the best, capped at 128.  "SMs" = CUs x resident workgroups.
int num_splits_heuristic(int work_blocks, int slots, int n_blocks, int max_splits) {
    if (work_blocks >= 0.8f * slots) return 1;
    max_splits = std::min(std::min(max_splits, slots), n_blocks);
    if (max_splits <= 1) return 1;
    auto cdiv = [](int a, int b) { return (a + b - 1) / b; };
    std::vector<float> eff(max_splits + 1, 0.f);
    float best = 0.f;
    for (int s = 1; s <= max_splits; ++s) {
        if (s > 1 && cdiv(n_blocks, s) == cdiv(n_blocks, s - 1)) continue;
        float waves = float(work_blocks * s) / slots;
        eff[s] = waves / std::ceil(waves);
        best = std::max(best, eff[s]);
    }
    for (int s = 1; s <= max_splits; ++s) {
        if (s > 1 && cdiv(n_blocks, s) == cdiv(n_blocks, s - 1)) continue;
        if (eff[s] >= 0.85f * best) return s;
    }
    return 1;
}

int hd_bucket(int d) { return d <= 64 ? 64 : (d <= 128 ? 128 : 256); }

hipError_t dispatch_fwd(const FwdParams& p, bool bf16, hipStream_t st) {
    const int hd = hd_bucket(p.d);
    if (hd == 64) return bf16 ? launch_fwd_hd64_bf16(p, st) : launch_fwd_hd64_f16(p, st);
    if (hd == 128) return bf16 ? launch_fwd_hd128_bf16(p, st) : launch_fwd_hd128_f16(p, st);
    if (hd == 256) return bf16 ? launch_fwd_hd256_bf16(p, st) : launch_fwd_hd256_f16(p, st);
    return hipErrorInvalidValue;
}

hipError_t dispatch_bwd(const BwdParams& p, bool bf16, hipStream_t st) {
    const int hd = hd_bucket(p.d);
    if (hd == 64) return bf16 ? launch_bwd_hd64_bf16(p, st) : launch_bwd_hd64_f16(p, st);
    if (hd == 128) return bf16 ? launch_bwd_hd128_bf16(p, st) : launch_bwd_hd128_f16(p, st);
    if (hd == 256) return bf16 ? launch_bwd_hd256_bf16(p, st) : launch_bwd_hd256_f16(p, st);
    return hipErrorInvalidValue;
}

// Score scaling as set_params_fprop_strided (paged_attn.cpp:93-102): with softcap the
// kernel computes tanh(s * scale / cap) and then scales by cap.
void set_scales(FwdParams& p, float softmax_scale, float softcap) {
    float scale_softmax;
    if (softcap > 0.f) { p.softcap_pre = softmax_scale / softcap; scale_softmax = softcap; }
    else { p.softcap_pre = 0.f; scale_softmax = softmax_scale; }
    p.scale_log2 = scale_softmax * 1.4426950408889634f;
    p.alibi_mul = 1.f / scale_softmax;
}

// Window normalisation (paged_attn.cpp:116-120): causal <=> wl < 0 && wr == 0.
template <typename P>
static LseAlibiParams lse_alibi_params(const P& p, float sign) {
    LseAlibiParams a{};
    a.src = p.lse; a.dst = nullptr; a.sign = sign;
    a.alibi = p.alibi; a.alibi_bstride = p.alibi_bstride;
    a.b = p.b; a.h = p.h; a.seqlen_q = p.seqlen_q; a.seqlen_k = p.seqlen_k;
    a.cu_seqlens_q = p.cu_seqlens_q; a.cu_seqlens_k = p.cu_seqlens_k;
    a.lse_batch = p.lse_batch; a.lse_head = p.lse_head;
    return a;
}
static LseAlibiParams lse_alibi_params(const FwdParams& p, float sign) {
    LseAlibiParams a = lse_alibi_params<FwdParams>(p, sign);
    a.dst = p.lse;
    a.seqused_k = p.seqused_k; a.leftpad_k = p.leftpad_k;
    return a;
}

// Returns the reference's is_causal (before the normalisation), which picks its ALiBi form.
bool set_windows(int& wl, int& wr, int seqlen_k) {
    const bool causal = wl < 0 && wr == 0;
    if (wl < 0 && wr >= 0) wl = seqlen_k;
    if (wl >= 0 && wr < 0) wr = seqlen_k;
    return causal;
}

bool check_common(const void* q, const void* k, const void* v, const void* o, int b, int h,
                  int hk, int d) {
    if (!q || !k || !v || !o) return fail(1, "q/k/v/o must be non-null device pointers");
    if (b <= 0) return fail(1, "batch size must be positive (got %d)", b);
    if (h <= 0 || hk <= 0 || h % hk != 0)
        return fail(1, "Number of heads in key/value must divide number of heads in query (h=%d, hk=%d)", h, hk);
    if (d <= 0 || d % 8 != 0) return fail(1, "head_size must be a positive multiple of 8 (got %d)", d);
    if (d > 256) return fail(1, "FlashAttention forward only supports head dimension at most 256 (got %d)", d);
    // the kernels move 16-byte chunks (b128 buffer loads, LDS-DMA, 16-byte stores)
    if (((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) & 15)
        return fail(1, "q/k/v/o must be 16-byte aligned device pointers");
    return true;
}

void dense_strides(FwdParams& p, int sq, int sk, int h, int hk, int d) {
    p.q_row = (int64_t)h * d;  p.q_head = d; p.q_batch = (int64_t)sq * h * d;
    p.k_row = (int64_t)hk * d; p.k_head = d; p.k_batch = (int64_t)sk * hk * d;
    p.v_row = (int64_t)hk * d; p.v_head = d; p.v_batch = (int64_t)sk * hk * d;
    p.o_row = (int64_t)h * d;  p.o_head = d; p.o_batch = (int64_t)sq * h * d;
    p.lse_batch = (int64_t)h * sq; p.lse_head = sq;
}

// Split scratch + launch (shared by every forward entry).
// Dropout RNG state of the calling thread (fmha_set_rng_state); read by every forward /
// backward call with p_dropout > 0.
thread_local uint64_t g_seed = 0, g_offset = 0;
// fmha_set_rng_state_device: the key read on the device (graph capture), and where a forward
// writes the key it used
thread_local const int64_t* g_seed_ptr = nullptr;
thread_local const int64_t* g_offset_ptr = nullptr;
thread_local uint64_t g_offset_add = 0;
thread_local int64_t* g_rng_out = nullptr;
// The device key is consumed by the next compute entry whatever its outcome (a call that fails
// validation before set_dropout must not leave a stale rng_out for a later one)
struct DevRngScope {
    ~DevRngScope() {
        g_seed_ptr = g_offset_ptr = nullptr;
        g_rng_out = nullptr;
    }
};

template <typename P>
bool set_dropout(P& p, float p_dropout, float softcap) {
    if (!(p_dropout >= 0.f && p_dropout < 1.f)) return fail(1, "p_dropout must be in [0, 1) (got %g)", p_dropout);
    // the reference's rule (export.cpp:515,737; flash_api_hip.cpp:400,606,895,1128)
    if (softcap > 0.f && p_dropout > 0.f) return fail(1, "Softcapping does not support dropout for now");
    p.drop = p_dropout > 0.f;
    if (!p.drop) return true;
    const float keep = 1.f - p_dropout;                   // paged_attn.cpp:106-113
    p.keep_thr = (uint32_t)std::floor(keep * 255.0);
    p.rp_keep = 1.f / keep;
    p.seed = g_seed;
    p.offset = g_seed_ptr ? g_offset_add : g_offset;
    p.seed_ptr = g_seed_ptr;
    p.offset_ptr = g_offset_ptr;
    p.rng_out = g_rng_out;
    return true;
}

// return_softmax: the dropped-out softmax [b, h, round128(sq), round128(sk)] after the forward
void run_sdmask(const FwdParams& p, void* s, bool bf16, hipStream_t st) {
    const int sq_r = (p.seqlen_q + 127) / 128 * 128, sk_r = (p.seqlen_k + 127) / 128 * 128;
    hip_ok(bf16 ? launch_sdmask_bf16(p, s, sq_r, sk_r, st) : launch_sdmask_f16(p, s, sq_r, sk_r, st),
           "return_softmax launch");
}

void run_fwd(FwdParams& p, bool bf16, hipStream_t st, int num_splits_req) {
    Options& o = options();
    p.device = current_device();
    p.num_cus = num_cus(p.device);
    p.waves = o.fwd_waves.load();
    p.fwd4 = o.fwd_w4.load();
    p.persist_per_cu = o.fwd_persistent.load();
    p.order = o.fwd_order.load();
    p.xcdq = o.fwd_xcdq.load();
    p.prio_hi = o.fwd_prio.load();
    p.pipe = o.fwd_pipe.load();
    p.max_slack = (float)o.fwd_slack.load();
    const int n_blocks = (p.seqlen_k + kBlockN - 1) / kBlockN;
    if (p.drop) num_splits_req = 1;       // no split-KV with dropout (paged_attn.cpp:180)
    int splits = num_splits_req;
    // Decode: the whole GQA group of query rows fits one 32-row MFMA tile -> the split-KV
    // decode kernel (every wave a split, fmha_decode_kernel.h); splits a multiple of 4.
    p.decode = o.fwd_decode.load() && !p.drop && !p.cu_seqlens_q && !p.cu_seqlens_k &&
               p.seqlen_q * p.group <= 32 && hd_bucket(p.d) == p.d && p.d <= 128 &&
               (!p.block_table || p.page_size % 16 == 0);
    if (p.decode) {
        const int tiles = (p.seqlen_k + 31) / 32;
        const int work = p.b * p.hk;
        int zs = num_splits_req > 0 ? (num_splits_req + 3) / 4
                                    : (o.dec_wg_per_cu.load() * p.num_cus + work - 1) / work;
        zs = std::max(1, std::min(zs, std::max(1, tiles / 8)));
        zs = std::min(zs, 32);
        splits = 4 * zs;
        // head-major workgroups (4 or 8 kv heads of one split) when the kv heads divide evenly
        const int hm = o.dec_hmaj.load();
        p.dec_mr = (o.dec_mr.load() == 16 && p.seqlen_q * p.group <= 16) ? 16 : 32;
        p.dec_hmaj = (hm == 2 && p.hk % 8 == 0) ? 2 : (hm >= 1 && p.hk % 4 == 0) ? 1 : 0;
    } else if (p.cu_seqlens_q) {
        splits = 1;  // varlen: single pass (the reference forces it too)
    } else if (splits <= 0) {
        const int work = p.b * p.hk * fwd_num_m_blocks(p.seqlen_q, p.group, p.d, p.waves);
        splits = num_splits_heuristic(work, p.num_cus * 2, n_blocks, 128);
    }
    if (!p.decode) splits = std::max(1, std::min(splits, std::min(128, std::max(1, n_blocks))));
    p.num_splits = splits;
    g_last_splits = splits;
    g_last_kernel[0] = 0;
    // Ragged caches (per-sequence lengths): the b * splits slots of a kv-head group are shared
    // in proportion to the sequences' key tiles, up to 128 splits for one sequence
    // (fmha_decode_kernel.h dec_slot); equal lengths give the same splits as without.
    p.dec_bal = p.decode && o.dec_bal.load() && !o.dec_fold.load() && p.dec_hmaj >= 1 &&
                p.seqused_k && p.b >= 2 && p.b <= 64;
    p.dec_slots = p.dec_bal ? p.b * splits : 0;
    p.dec_cap = p.dec_bal ? std::min(p.dec_slots, 128) : 0;
    p.dec_ns = nullptr;
    p.comb_row = o.comb_row.load();
    const int ext = p.dec_bal ? p.dec_cap : splits;   // split extent of the scratch
    if (splits > 1) {
        const int hd = hd_bucket(p.d);
        const size_t rows = (size_t)p.b * p.h * p.seqlen_q;
        const size_t obytes = (size_t)ext * rows * hd * sizeof(float);
        const size_t lbytes = (size_t)ext * rows * sizeof(float);
        const size_t bytes = obytes + lbytes + (p.dec_bal ? (size_t)p.b * sizeof(int) : 0);
        char* base = (char*)pool_get(st, bytes);
        if (!base) { fail(3, "could not allocate %zu bytes of split scratch", bytes); return; }
        p.oaccum = (float*)base;
        p.lseaccum = (float*)(base + obytes);
        if (p.dec_bal) p.dec_ns = (int*)(base + obytes + lbytes);
    }
    p.dec_ctr = nullptr;
    if (p.decode && o.dec_fold.load()) {
        p.dec_ctr = dec_counters(st, p.b * p.hk);
        if (!p.dec_ctr) { fail(3, "could not allocate the decode split counters"); return; }
    }
    // dynamic item queue: ragged (varlen) row blocks balance across CUs as they finish; also the
    // dense D = 128 launches without a right window (the 16x16x32 ping-pong body), whose equal
    // items ran 0.7-1.0 % faster from the per-XCD queues than from the static XCD pairs on two
    // leases (causal launches keep the pairs, which balance their item sizes),
    // and the D = 128 launches with a left window, whose row blocks past the window's width all
    // carry the same work, so the pairs unbalance them (+7 % at (1023, 0), +4 % at (255, 0);
    // profiles/r06_window_dyn_ab.log), and the non-causal ALiBi launches (32x32x16 body, +0.5 to
    // +3.2 % on two boxes; non-causal softcap measured -0.4 % and keeps the pairs:
    // r06_noncausal_feat_ab.log)
    p.work_ctr = nullptr;
    const int dyn = o.fwd_dyn.load();
    const bool nc16 = p.d == 128 && p.wr < 0 && p.fwd4 == 4 && !p.alibi && !(p.softcap_pre > 0.f);
    const bool ncab = p.d == 128 && p.wr < 0 && p.fwd4 == 4 && p.alibi;
    const bool win = p.d == 128 && p.fwd4 == 4 && p.wl >= 0 && p.wl < p.seqlen_k;  // causal: wl = seqlen_k
    if (!p.decode && splits == 1 && (dyn == 2 || (dyn == 1 && (p.cu_seqlens_q || nc16 || ncab || win)))) {
        p.work_ctr = counter_get(st);
        if (!p.work_ctr) { fail(3, "could not allocate the item-queue counters"); return; }
    }
    if (!hip_ok(dispatch_fwd(p, bf16, st), "forward launch")) return;
    // causal ALiBi: the LSE in the reference's convention (+slope key, mask_hip.h:163-164)
    if (p.lse && p.alibi && p.alibi_causal) hip_ok(launch_lse_alibi(lse_alibi_params(p, +1.f), st), "LSE ALiBi pass");
}

}  // namespace

extern "C" {

const char* fmha_last_error(void) { return g_err.c_str(); }
int fmha_last_status(void) { return g_status; }
int fmha_last_num_splits(void) { return g_last_splits; }
const char* fmha_last_kernel(void) { return g_last_kernel; }
const char* fmha_version(void) { return XFA_VARIANTS ? "xf-fmha-gfx950 2.4 (variants)" : "xf-fmha-gfx950 2.4"; }

void fmha_set_rng_state(uint64_t seed, uint64_t offset) {
    g_seed = seed;
    g_offset = offset;
    g_seed_ptr = g_offset_ptr = nullptr;
    g_rng_out = nullptr;
}

void fmha_set_rng_state_device(const int64_t* seed_ptr, const int64_t* offset_ptr, uint64_t offset_add,
                               int64_t* rng_out) {
    g_seed_ptr = (seed_ptr && offset_ptr) ? seed_ptr : nullptr;
    g_offset_ptr = g_seed_ptr ? offset_ptr : nullptr;
    g_offset_add = offset_add;
    g_rng_out = rng_out;
}

int fmha_set_option(const char* name, int value) {
    clear_error();
    if (!name) { fail(1, "option name is null"); return -1; }
    Options& o = options();
    struct Knob { const char* name; std::atomic<int>* slot; int lo, hi; };
    const Knob knobs[] = {
        {"fwd_waves", &o.fwd_waves, 4, 8},       {"fwd_prio", &o.fwd_prio, 0, 1},
        {"fwd_persistent", &o.fwd_persistent, 0, 8}, {"fwd_slack", &o.fwd_slack, 0, 16},
        {"fwd_order", &o.fwd_order, 0, 1},       {"fwd_dyn", &o.fwd_dyn, 0, 2},
        {"fwd_xcdq", &o.fwd_xcdq, 0, 1},         {"fwd_pipe", &o.fwd_pipe, 0, 2},
        {"fwd_decode", &o.fwd_decode, 0, 1},     {"dec_wg_per_cu", &o.dec_wg_per_cu, 1, 16},
        {"dec_hmaj", &o.dec_hmaj, 0, 2},
        {"dec_mr", &o.dec_mr, 16, 32},           {"fwd_w4", &o.fwd_w4, 0, 4},
        {"bwd_order", &o.bwd_order, 0, 1},       {"bwd_desc", &o.bwd_desc, 0, 1},
        {"dec_fold", &o.dec_fold, 0, 1},        {"dec_bal", &o.dec_bal, 0, 1},
        {"fp8_w4", &o.fp8_w4, 0, 2},           {"comb_row", &o.comb_row, 0, 1},
    };
    for (const Knob& k : knobs) {
        if (strcmp(name, k.name)) continue;
        if (value < k.lo || value > k.hi || (k.slot == &o.fwd_waves && value != 4 && value != 8) ||
            (k.slot == &o.dec_mr && value != 16 && value != 32)) {
            fail(1, "option %s: value %d out of range [%d, %d]", name, value, k.lo, k.hi);
            return -1;
        }
        if (!XFA_VARIANTS && ((k.slot == &o.fwd_w4 && value == 1) || (k.slot == &o.fp8_w4 && value == 2))) {
            fail(1, "option %s = %d selects a kernel only the variants build has "
                    "(lib/variants/libpaged-attention.so, build.py --variants)", name, value);
            return -1;
        }
        k.slot->store(value);
        return 0;
    }
    fail(1, "unknown option '%s'", name);
    return -1;
}

int fmha_get_option(const char* name) {
    clear_error();
    Options& o = options();
    if (!name) { fail(1, "option name is null"); return -1; }
#define XFA_GET(n) if (!strcmp(name, #n)) return o.n.load();
    XFA_GET(fwd_waves) XFA_GET(fwd_prio) XFA_GET(fwd_persistent) XFA_GET(fwd_slack)
    XFA_GET(fwd_order) XFA_GET(fwd_dyn) XFA_GET(fwd_xcdq) XFA_GET(fwd_pipe) XFA_GET(fwd_decode)
    XFA_GET(dec_wg_per_cu) XFA_GET(dec_hmaj) XFA_GET(dec_mr) XFA_GET(fwd_w4)
    XFA_GET(bwd_order) XFA_GET(bwd_desc) XFA_GET(dec_fold) XFA_GET(dec_bal) XFA_GET(fp8_w4)
    XFA_GET(comb_row)
#undef XFA_GET
    fail(1, "unknown option '%s'", name);
    return -1;
}

void fmha_fwd(void* q_ptr, void* k_ptr, void* v_ptr, void* o_ptr, void* alibi_slopes_ptr,
              const int32_t seqlen_q, const int32_t seqlen_k, const int32_t batch_size,
              const int32_t num_heads, const int32_t num_heads_k, const int32_t head_size,
              const float p_dropout, hipStream_t stream, hipDeviceProp_t* /*dprops*/,
              const float softmax_scale, void* p_ptr, void* softmax_lse_ptr,
              int window_size_left, int window_size_right, const float softcap,
              const bool return_softmax, bool is_fp16, int num_splits) {
    try {
        begin_fwd();
        DevRngScope rng_scope;
        if (!check_common(q_ptr, k_ptr, v_ptr, o_ptr, batch_size, num_heads, num_heads_k, head_size)) return;
        REQUIRE(seqlen_q > 0 && seqlen_k > 0, "seqlen_q/seqlen_k must be positive (%d, %d)", seqlen_q, seqlen_k);
        REQUIRE(!return_softmax || p_dropout > 0.f, "return_softmax is only supported when p_dropout > 0.0");
        REQUIRE(!return_softmax || (p_ptr && softmax_lse_ptr), "return_softmax needs the p and softmax_lse buffers");
        if (!slab_ok("q/o", seqlen_q, (int64_t)num_heads * head_size, 2) ||
            !slab_ok("k/v", seqlen_k, (int64_t)num_heads_k * head_size, 2)) return;
        FwdParams p{};
        p.q = q_ptr; p.k = k_ptr; p.v = v_ptr; p.o = o_ptr;
        p.lse = (float*)softmax_lse_ptr;
        dense_strides(p, seqlen_q, seqlen_k, num_heads, num_heads_k, head_size);
        p.b = batch_size; p.h = num_heads; p.hk = num_heads_k; p.group = num_heads / num_heads_k;
        p.d = head_size; p.seqlen_q = seqlen_q; p.seqlen_k = seqlen_k;
        p.alibi_causal = set_windows(window_size_left, window_size_right, seqlen_k);
        p.wl = window_size_left; p.wr = window_size_right;
        set_scales(p, softmax_scale, softcap);
        p.alibi = (const float*)alibi_slopes_ptr;
        p.alibi_bstride = batch_size > 1 ? num_heads : 0;   // paged_attn.cpp:375
        if (!set_dropout(p, p_dropout, softcap)) return;
        run_fwd(p, !is_fp16, stream, num_splits);
        if (return_softmax && g_status == 0) run_sdmask(p, p_ptr, !is_fp16, stream);
    } catch (...) {
        fail(9, "internal error in fmha_fwd");
    }
}

void fmha_fwd_strided(void* q, void* k, void* v, void* o, void* alibi_slopes, void* softmax_lse,
                      int32_t seqlen_q, int32_t seqlen_k, int32_t batch_size, int32_t num_heads,
                      int32_t num_heads_k, int32_t head_size, const int64_t* st,
                      float softmax_scale, int window_size_left, int window_size_right,
                      float softcap, bool is_fp16, int num_splits, hipStream_t stream,
                      float p_dropout, void* s_dmask) {
    try {
        begin_fwd();
        DevRngScope rng_scope;
        if (!check_common(q, k, v, o, batch_size, num_heads, num_heads_k, head_size)) return;
        REQUIRE(st != nullptr, "strides must be non-null");
        REQUIRE(seqlen_q > 0 && seqlen_k > 0, "seqlen_q/seqlen_k must be positive (%d, %d)", seqlen_q, seqlen_k);
        for (int i = 0; i < 12; ++i) REQUIRE(st[i] >= 0, "strides must be non-negative");
        {   // (a stride over an extent of 1 is never applied)
            const int ext[12] = {batch_size, seqlen_q, num_heads, batch_size, seqlen_k, num_heads_k,
                                 batch_size, seqlen_k, num_heads_k, batch_size, seqlen_q, num_heads};
            for (int i = 0; i < 12; ++i)
                REQUIRE(ext[i] == 1 || st[i] % 8 == 0,
                        "strides must be multiples of 8 elements (16 bytes): stride %d is %lld", i,
                        (long long)st[i]);
        }
        // one sequence's slab of each tensor, addressed with 32-bit offsets by the kernels
        auto slab = [&](const char* what, int rows, int64_t row, int64_t head, int heads) {
            const int64_t bytes = ((int64_t)(rows - 1) * row + (int64_t)(heads - 1) * head + head_size) * 2;
            if (bytes < kMaxSlabBytes) return true;
            return fail(1, "%s: one sequence spans %lld bytes; this build addresses a sequence with "
                        "32-bit offsets and supports < %lld bytes", what, (long long)bytes,
                        (long long)kMaxSlabBytes);
        };
        if (!slab("q", seqlen_q, st[1], st[2], num_heads) || !slab("k", seqlen_k, st[4], st[5], num_heads_k) ||
            !slab("v", seqlen_k, st[7], st[8], num_heads_k) || !slab("o", seqlen_q, st[10], st[11], num_heads)) return;
        FwdParams p{};
        p.q = q; p.k = k; p.v = v; p.o = o;
        p.lse = (float*)softmax_lse;
        p.q_batch = st[0]; p.q_row = st[1]; p.q_head = st[2];
        p.k_batch = st[3]; p.k_row = st[4]; p.k_head = st[5];
        p.v_batch = st[6]; p.v_row = st[7]; p.v_head = st[8];
        p.o_batch = st[9]; p.o_row = st[10]; p.o_head = st[11];
        p.lse_batch = (int64_t)num_heads * seqlen_q; p.lse_head = seqlen_q;
        p.b = batch_size; p.h = num_heads; p.hk = num_heads_k; p.group = num_heads / num_heads_k;
        p.d = head_size; p.seqlen_q = seqlen_q; p.seqlen_k = seqlen_k;
        p.alibi_causal = set_windows(window_size_left, window_size_right, seqlen_k);
        p.wl = window_size_left; p.wr = window_size_right;
        set_scales(p, softmax_scale, softcap);
        p.alibi = (const float*)alibi_slopes;
        p.alibi_bstride = batch_size > 1 ? num_heads : 0;
        REQUIRE(!s_dmask || (p_dropout > 0.f && softmax_lse), "s_dmask needs p_dropout > 0 and softmax_lse");
        if (!set_dropout(p, p_dropout, softcap)) return;
        run_fwd(p, !is_fp16, stream, num_splits);
        if (s_dmask && g_status == 0) run_sdmask(p, s_dmask, !is_fp16, stream);
    } catch (...) {
        fail(9, "internal error in fmha_fwd_strided");
    }
}

void fmha_fwd_fp8(void* q, void* k, void* v, void* o, void* softmax_lse, float q_scale,
                  float k_scale, float v_scale, int32_t seqlen_q, int32_t seqlen_k,
                  int32_t batch_size, int32_t num_heads, int32_t num_heads_k, int32_t head_size,
                  float softmax_scale, int window_size_left, int window_size_right, bool out_fp16,
                  hipStream_t stream) {
    try {
        begin_fwd();
        if (!check_common(q, k, v, o, batch_size, num_heads, num_heads_k, head_size)) return;
        REQUIRE(head_size == 128, "the fp8 forward supports head_size 128 (got %d)", head_size);
        REQUIRE(seqlen_q > 0 && seqlen_k > 0, "seqlen_q/seqlen_k must be positive (%d, %d)", seqlen_q, seqlen_k);
        REQUIRE(q_scale > 0.f && k_scale > 0.f && v_scale > 0.f, "fp8 descales must be positive");
        if (!slab_ok("q", seqlen_q, (int64_t)num_heads * head_size, 1) ||
            !slab_ok("k/v", seqlen_k, (int64_t)num_heads_k * head_size, 1) ||
            !slab_ok("o", seqlen_q, (int64_t)num_heads * head_size, 2)) return;
        FwdParams p{};
        p.q = q; p.k = k; p.v = v; p.o = o;
        p.lse = (float*)softmax_lse;
        // element strides; fp8 elements are bytes, so q/k/v strides are byte strides too
        dense_strides(p, seqlen_q, seqlen_k, num_heads, num_heads_k, head_size);
        p.b = batch_size; p.h = num_heads; p.hk = num_heads_k; p.group = num_heads / num_heads_k;
        p.d = head_size; p.seqlen_q = seqlen_q; p.seqlen_k = seqlen_k;
        p.alibi_causal = set_windows(window_size_left, window_size_right, seqlen_k);
        p.wl = window_size_left; p.wr = window_size_right;
        set_scales(p, softmax_scale, 0.f);
        p.q_scale = q_scale; p.k_scale = k_scale; p.v_scale = v_scale;
        Options& op = options();
        p.device = current_device();
        p.num_cus = num_cus(p.device);
        p.persist_per_cu = op.fwd_persistent.load();
        p.order = op.fwd_order.load();
        p.max_slack = (float)op.fwd_slack.load();
        p.num_splits = 1;
        p.fwd4 = op.fp8_w4.load();
        p.xcdq = op.fwd_xcdq.load();
        // fwd_dyn = 2: the dynamic per-XCD item queues for the dense fp8 launch too
        p.work_ctr = nullptr;
        if (op.fwd_dyn.load() == 2) {
            p.work_ctr = counter_get(stream);
            REQUIRE(p.work_ctr, "could not allocate the item-queue counters");
        }
        g_last_splits = 1;
        g_last_kernel[0] = 0;
        hip_ok(launch_fwd_fp8(p, out_fp16, stream), "fp8 forward launch");
    } catch (...) {
        fail(9, "internal error in fmha_fwd_fp8");
    }
}

void fmha_varlen_fwd_ex(void* q, void* k, void* v, void* o, void* softmax_lse,
                        void* cu_seqlens_q, void* cu_seqlens_k, void* seqused_k,
                        void* block_table, int32_t block_table_stride, int32_t page_block_size,
                        void* alibi_slopes, int32_t alibi_batch_stride,
                        int32_t max_seqlen_q, int32_t max_seqlen_k, int32_t total_q,
                        int32_t batch_size, int32_t num_heads, int32_t num_heads_k,
                        int32_t head_size, float softmax_scale, int window_size_left,
                        int window_size_right, float softcap, bool is_fp16, hipStream_t stream,
                        float p_dropout, void* s_dmask) {
    try {
        begin_fwd();
        DevRngScope rng_scope;
        if (!check_common(q, k, v, o, batch_size, num_heads, num_heads_k, head_size)) return;
        REQUIRE(cu_seqlens_q && (cu_seqlens_k || block_table),
                "cu_seqlens_q and cu_seqlens_k (or a block table) must be given");
        REQUIRE(max_seqlen_q > 0 && max_seqlen_k >= 0, "max_seqlen_q must be positive");
        if (max_seqlen_k == 0) { fail(1, "max_seqlen_k == 0: nothing to attend to"); return; }
        if (!slab_ok("q/o", max_seqlen_q, (int64_t)num_heads * head_size, 2) ||
            (!block_table && !slab_ok("k/v", max_seqlen_k, (int64_t)num_heads_k * head_size, 2))) return;
        FwdParams p{};
        p.q = q; p.k = k; p.v = v; p.o = o; p.lse = (float*)softmax_lse;
        const int h = num_heads, hk = num_heads_k, d = head_size;
        p.q_row = (int64_t)h * d; p.q_head = d; p.q_batch = 0;
        p.o_row = (int64_t)h * d; p.o_head = d; p.o_batch = 0;
        p.k_row = (int64_t)hk * d; p.k_head = d; p.k_batch = 0;
        p.v_row = (int64_t)hk * d; p.v_head = d; p.v_batch = 0;
        p.cu_seqlens_q = (const int*)cu_seqlens_q;
        if (block_table) {
            REQUIRE(page_block_size > 0, "page_block_size must be positive");
            p.block_table = (const int*)block_table;
            p.bt_stride = block_table_stride;
            p.page_size = page_block_size;
            p.k_batch = (int64_t)page_block_size * hk * d;
            p.v_batch = (int64_t)page_block_size * hk * d;
            // key lengths from seqused_k or cu_seqlens_k; pages are per sequence (no k offset)
            p.cu_seqlens_k = (const int*)cu_seqlens_k;
            REQUIRE(seqused_k || cu_seqlens_k, "paged varlen needs seqused_k or cu_seqlens_k");
        } else {
            p.cu_seqlens_k = (const int*)cu_seqlens_k;
        }
        p.seqused_k = (const int*)seqused_k;
        p.b = batch_size; p.h = h; p.hk = hk; p.group = h / hk; p.d = d;
        p.seqlen_q = max_seqlen_q; p.seqlen_k = max_seqlen_k;
        p.alibi_causal = set_windows(window_size_left, window_size_right, max_seqlen_k);
        p.wl = window_size_left; p.wr = window_size_right;
        set_scales(p, softmax_scale, softcap);
        p.alibi = (const float*)alibi_slopes; p.alibi_bstride = alibi_batch_stride;
        // unpadded LSE [num_heads, total_q] (export.cpp:827): index = h*total_q + q_off + pos
        p.lse_batch = 0;
        p.lse_head = total_q;
        REQUIRE(!softmax_lse || total_q > 0, "total_q must be given to address the LSE");
        REQUIRE(!s_dmask || (p_dropout > 0.f && softmax_lse && !block_table),
                "s_dmask needs p_dropout > 0, softmax_lse and a non-paged K/V");
        REQUIRE(p_dropout == 0.f || !block_table, "dropout over a paged K/V cache is not supported");
        if (!set_dropout(p, p_dropout, softcap)) return;
        run_fwd(p, !is_fp16, stream, 1);
        if (s_dmask && g_status == 0) run_sdmask(p, s_dmask, !is_fp16, stream);
    } catch (...) {
        fail(9, "internal error in fmha_varlen_fwd_ex");
    }
}

void fmha_varlen_fwd(void* q_ptrs, void* k_ptrs, void* v_ptrs, void* o_ptrs,
                     void* cu_seqlens_q_ptrs, void* cu_seqlens_k_ptrs,
                     const int32_t max_seqlen_q, const int32_t max_seqlen_k,
                     const int32_t batch_size, const int32_t num_heads,
                     const int32_t num_heads_k, const int32_t head_size, hipStream_t stream,
                     const float softmax_scale, const bool /*is_causal*/, const bool is_fp16,
                     int window_size_left, int window_size_right) {
    fmha_varlen_fwd_ex(q_ptrs, k_ptrs, v_ptrs, o_ptrs, nullptr, cu_seqlens_q_ptrs,
                       cu_seqlens_k_ptrs, nullptr, nullptr, 0, 0, nullptr, 0, max_seqlen_q,
                       max_seqlen_k, 0, batch_size, num_heads, num_heads_k, head_size,
                       softmax_scale, window_size_left, window_size_right, 0.f, is_fp16, stream,
                       0.f, nullptr);
}

void fmha_page_kvcache_fwd_ex(void* q, void* kcache, void* vcache, void* o, void* softmax_lse,
                              void* block_table, int32_t block_table_stride, void* cache_seqlens,
                              int32_t seqlen_q, int32_t max_seqlen_k, int32_t batch_size,
                              int32_t num_heads, int32_t num_heads_k, int32_t head_size,
                              int32_t page_block_size, float softmax_scale,
                              int window_size_left, int window_size_right, float softcap,
                              void* alibi_slopes, int32_t alibi_batch_stride, int32_t num_splits,
                              int32_t kv_dtype, float k_scale, float v_scale,
                              void* cache_leftpad, bool is_fp16, hipStream_t stream) {
    try {
        begin_fwd();
        if (!check_common(q, kcache, vcache, o, batch_size, num_heads, num_heads_k, head_size)) return;
        REQUIRE(block_table, "block_table must be given for the paged KV path");
        REQUIRE(page_block_size > 0, "page_block_size must be positive");
        REQUIRE(seqlen_q > 0 && max_seqlen_k > 0, "seqlen_q / seqlen_k must be positive");
        REQUIRE(kv_dtype == 0 || kv_dtype == 1, "kv_dtype must be 0 (same as q) or 1 (fp8 e4m3fn)");
        REQUIRE(block_table_stride > 0, "block_table_stride must be positive");
        // export.cpp:1627-1628 (commented out in the reference): no paged KV with leftpad
        REQUIRE(!cache_leftpad || max_seqlen_k <= page_block_size,
                "cache_leftpad needs a non-paged cache (one page per sequence): Paged KV and "
                "leftpad_k are not supported at the same time");
        if (!slab_ok("q/o", seqlen_q, (int64_t)num_heads * head_size, 2) ||
            !slab_ok("kcache/vcache page", page_block_size, (int64_t)num_heads_k * head_size, kv_dtype == 1 ? 1 : 2)) return;
        FwdParams p{};
        const int h = num_heads, hk = num_heads_k, d = head_size;
        p.q = q; p.k = kcache; p.v = vcache; p.o = o; p.lse = (float*)softmax_lse;
        dense_strides(p, seqlen_q, max_seqlen_k, h, hk, d);
        p.k_batch = (int64_t)page_block_size * hk * d;   // page stride (paged_attn.cpp:506-507)
        p.v_batch = (int64_t)page_block_size * hk * d;
        p.block_table = (const int*)block_table;
        p.bt_stride = block_table_stride;
        p.page_size = page_block_size;
        p.seqused_k = (const int*)cache_seqlens;         // non-cumulative (paged_attn.cpp:518-519)
        p.leftpad_k = (const int*)cache_leftpad;
        p.b = batch_size; p.h = h; p.hk = hk; p.group = h / hk; p.d = d;
        p.seqlen_q = seqlen_q; p.seqlen_k = max_seqlen_k;
        p.alibi_causal = set_windows(window_size_left, window_size_right, max_seqlen_k);
        p.wl = window_size_left; p.wr = window_size_right;
        set_scales(p, softmax_scale, softcap);
        p.alibi = (const float*)alibi_slopes; p.alibi_bstride = alibi_batch_stride;
        p.kv_fp8 = kv_dtype == 1; p.k_scale = k_scale; p.v_scale = v_scale;
        run_fwd(p, !is_fp16, stream, num_splits);
    } catch (...) {
        fail(9, "internal error in fmha_page_kvcache_fwd_ex");
    }
}

void fmha_kvcache_append(void* q, void* q_out, void* kcache, void* vcache, const void* knew,
                         const void* vnew, int32_t seqlen_new, const void* block_table,
                         int32_t block_table_stride, int32_t page_block_size,
                         const void* cache_seqlens, void* seqlens_out, const void* rotary_cos,
                         const void* rotary_sin, int32_t rotary_dim, bool is_rotary_interleaved,
                         bool q_rotary_per_token, int32_t batch_size, int32_t seqlen_q,
                         int32_t num_heads, int32_t num_heads_k, int32_t head_size,
                         bool is_fp16, hipStream_t stream) {
    try {
        clear_error();
        REQUIRE(kcache && vcache && block_table && cache_seqlens,
                "kcache, vcache, block_table and cache_seqlens must be given");
        REQUIRE(seqlen_new >= 0, "seqlen_new must be >= 0");
        REQUIRE(seqlen_new == 0 || (knew && vnew), "new K and V must both be given");
        REQUIRE(batch_size > 0 && num_heads > 0 && num_heads_k > 0 && num_heads % num_heads_k == 0,
                "invalid batch / head counts");
        REQUIRE(head_size > 0 && head_size % 8 == 0 && head_size <= 256,
                "head_size must be a multiple of 8 (<= 256) for the append pass");
        REQUIRE(page_block_size > 0, "page_block_size must be positive");
        REQUIRE(block_table_stride > 0, "block_table_stride must be positive");
        // the kernel reads cache_seqlens while writing seqlens_out: in-place is a race
        REQUIRE(seqlens_out != cache_seqlens, "seqlens_out must not alias cache_seqlens");
        REQUIRE(rotary_dim >= 0 && rotary_dim <= head_size && rotary_dim % 16 == 0,
                "Only rotary dimensions divisible by 16 and <= headdim are supported");
        REQUIRE(rotary_dim == 0 || (rotary_cos && rotary_sin && q && q_out),
                "rotary needs cos, sin, q and q_out");
        AppendParams p{};
        p.q = q; p.q_out = q_out; p.kcache = kcache; p.vcache = vcache;
        p.knew = knew; p.vnew = vnew;
        p.block_table = (const int*)block_table; p.bt_stride = block_table_stride;
        p.page = page_block_size;
        p.cache_seqlens = (const int*)cache_seqlens; p.seqlens_out = (int*)seqlens_out;
        p.cos = rotary_cos; p.sin = rotary_sin; p.rdim = rotary_dim;
        p.interleaved = is_rotary_interleaved; p.q_per_token = q_rotary_per_token;
        p.b = batch_size; p.sq = seqlen_q; p.h = num_heads; p.hk = num_heads_k; p.d = head_size;
        p.snew = seqlen_new;
        p.q_head = head_size; p.q_row = (int64_t)num_heads * head_size;
        p.q_batch = (int64_t)seqlen_q * p.q_row;
        p.kn_head = head_size; p.kn_row = (int64_t)num_heads_k * head_size;
        p.kn_batch = (int64_t)seqlen_new * p.kn_row;
        p.head_stride = head_size; p.row_stride = (int64_t)num_heads_k * head_size;
        p.page_stride = (int64_t)page_block_size * p.row_stride;
        hip_ok(launch_append(p, is_fp16, stream), "append launch");
    } catch (...) {
        fail(9, "internal error in fmha_kvcache_append");
    }
}

void fmha_page_kvcache_fwd(void* q_ptr, void* kcache_ptr, void* vcache_ptr, void* /*k_ptr*/,
                           void* /*v_ptr*/, void* o_ptr, void* block_table_ptr,
                           void* cache_seqlens_k_ptr, const int32_t max_cache_seq_k,
                           const int32_t seqlen_q, const int32_t seqlen_k,
                           const int32_t batch_size, const int32_t num_heads,
                           const int32_t num_heads_k, const int32_t head_size,
                           const int32_t page_block_size, hipStream_t stream,
                           const float softmax_scale, int window_size_left,
                           int window_size_right, const int32_t num_splits,
                           void* /*cache_batch_idx_ptr*/, void* /*rotary_cos_ptr*/,
                           void* /*rotary_sin_ptr*/, bool /*is_causal*/,
                           bool /*is_rotary_interleaved*/, bool is_fp16) {
    if (page_block_size <= 0) { begin_fwd(); fail(1, "page_block_size must be positive"); return; }
    fmha_page_kvcache_fwd_ex(q_ptr, kcache_ptr, vcache_ptr, o_ptr, nullptr, block_table_ptr,
                             max_cache_seq_k / page_block_size, cache_seqlens_k_ptr, seqlen_q,
                             seqlen_k, batch_size, num_heads, num_heads_k, head_size,
                             page_block_size, softmax_scale, window_size_left, window_size_right,
                             0.f, nullptr, 0, num_splits, 0, 1.f, 1.f, nullptr, is_fp16, stream);
}


// ------------------------------------------------------------------ backward -----------
// Workspace: fp32 dq_accum [tokens][h][HD] + fp32 D = rowsum(dO*O) [tokens][h].  Deterministic:
// S = min(ceil(CUs / (b * hk)), key blocks) dq_accum slices (the reference's bound,
// export.cpp:1090-1091, counts query heads: here a workgroup covers a kv head's whole GQA group,
// and no workgroup walks more slices than there are 256-key blocks), and at most what
// kDetSliceCap bytes of slices hold; workgroup (bh, s) adds key blocks s, s + S, ... into slice s
// in order.  Any S >= 1 is a valid schedule (bitwise reproducible for a given S), so a run whose
// workspace holds fewer slices than its device would pick uses as many as fit.
static int bwd_block_n_host(int d) { return hd_bucket(d) > 128 ? 128 : 256; }
static size_t bwd_acc_bytes(int64_t tokens, int h, int d) {
    return (((size_t)tokens * h * hd_bucket(d) * sizeof(float)) + 255) / 256 * 256;
}
static size_t bwd_dsum_bytes(int64_t tokens, int h) {
    return (((size_t)tokens * h * sizeof(float)) + 255) / 256 * 256;
}
constexpr size_t kDetSliceCap = (size_t)8 << 30;     // bytes of dQ slices beyond the first
static int bwd_slices(int64_t tokens, int batch, int h, int hk, int d, int seqlen_k, bool det) {
    if (!det) return 1;
    const int units = std::max(1, batch * hk);
    const int nkb = std::max(1, (seqlen_k + bwd_block_n_host(d) - 1) / bwd_block_n_host(d));
    int s = std::min(nkb, (num_cus(current_device()) + units - 1) / units);
    const size_t acc = std::max<size_t>(256, bwd_acc_bytes(tokens, h, d));
    s = (int)std::min<size_t>((size_t)s, 1 + kDetSliceCap / acc);
    return std::max(1, s);
}
// workspace: [dQ slices][D = rowsum(dO O)][lse_fix: the causal-ALiBi LSE in the kernels' form]
static size_t bwd_ws_bytes(int64_t tokens, int h, int d, int slices) {
    return (size_t)slices * bwd_acc_bytes(tokens, h, d) + 2 * bwd_dsum_bytes(tokens, h);
}
// causal ALiBi: softmax_lse (the reference's convention) -> lse_fix in the kernels' own, which
// the backward then reads
static bool bwd_lse_convention(BwdParams& p, hipStream_t st) {
    if (!(p.alibi && p.alibi_causal)) return true;
    LseAlibiParams a = lse_alibi_params(p, -1.f);
    a.dst = p.lse_fix;
    if (!hip_ok(launch_lse_alibi(a, st), "LSE ALiBi pass")) return false;
    p.lse = p.lse_fix;
    return true;
}
// slices a caller's workspace of `bytes` holds (0 if not even one)
static int bwd_slices_fit(int64_t tokens, int h, int d, size_t bytes) {
    const size_t fixed = 2 * bwd_dsum_bytes(tokens, h), acc = std::max<size_t>(1, bwd_acc_bytes(tokens, h, d));
    return bytes < fixed ? 0 : (int)std::min<size_t>((bytes - fixed) / acc, 1 << 20);
}

size_t fmha_bwd_workspace_size(int32_t seqlen_q, int32_t seqlen_k, int32_t batch_size,
                               int32_t num_heads, int32_t num_heads_k, int32_t head_size,
                               bool deterministic) {
    const int64_t tok = (int64_t)batch_size * seqlen_q;
    return bwd_ws_bytes(tok, num_heads, head_size,
                        bwd_slices(tok, batch_size, num_heads, num_heads_k, head_size, seqlen_k, deterministic));
}

size_t fmha_varlen_bwd_workspace_size(int32_t total_q, int32_t max_seqlen_k, int32_t batch_size,
                                      int32_t num_heads, int32_t num_heads_k, int32_t head_size,
                                      bool deterministic) {
    return bwd_ws_bytes(total_q, num_heads, head_size,
                        bwd_slices(total_q, batch_size, num_heads, num_heads_k, head_size, max_seqlen_k, deterministic));
}

// The pre / convert kernels index (token, head, 16-byte chunk) with one 32-bit thread id.
static bool bwd_rows_ok(int64_t tokens, int h, int d) {
    const int64_t threads = tokens * h * (hd_bucket(d) / 8);
    if (threads < (1LL << 31) - 256) return true;
    return fail(1, "backward: %lld (token, head) rows exceed the 32-bit thread index", (long long)(tokens * h));
}

static bool bwd_common(BwdParams& p, float softmax_scale, float softcap, int wl, int wr,
                       int seqlen_k_norm) {
    p.alibi_causal = set_windows(wl, wr, seqlen_k_norm);
    p.wl = wl; p.wr = wr;
    float scale_softmax = softmax_scale;
    p.softcap_on = softcap > 0.f;
    if (p.softcap_on) { p.softcap_pre = softmax_scale / softcap; scale_softmax = softcap; }
    p.scale = softmax_scale;
    p.scale_log2 = scale_softmax * 1.4426950408889634f;
    p.alibi_mul = 1.f / scale_softmax;
    p.device = current_device();
    p.order = options().bwd_order.load();
    p.desc = options().bwd_desc.load();
    return true;
}

void fmha_bwd(void* dout, void* q, void* k, void* v, void* out, void* softmax_lse, void* dq,
              void* dk, void* dv, void* alibi_slopes, void* softmax_d, int32_t seqlen_q,
              int32_t seqlen_k, int32_t batch_size, int32_t num_heads, int32_t num_heads_k,
              int32_t head_size, float p_dropout, float softmax_scale, int window_size_left,
              int window_size_right, float softcap, bool deterministic, bool is_fp16,
              hipStream_t stream, void* workspace, size_t workspace_bytes) {
    try {
        clear_error();
        DevRngScope rng_scope;
        if (!check_common(q, k, v, out, batch_size, num_heads, num_heads_k, head_size)) return;
        REQUIRE(head_size <= 256, "the backward supports head dimension at most 256 (got %d)", head_size);
        REQUIRE(dout && softmax_lse && dq && dk && dv, "dout/softmax_lse/dq/dk/dv must be non-null");
        REQUIRE(!(softcap > 0.f && p_dropout > 0.f), "Softcapping does not support dropout for now");
        REQUIRE(seqlen_q > 0 && seqlen_k > 0, "seqlen_q/seqlen_k must be positive");
        const int h = num_heads, hk = num_heads_k, d = head_size;
        if (!slab_ok("q/out/dout/dq", seqlen_q, (int64_t)h * d, 2) ||
            !slab_ok("k/v/dk/dv", seqlen_k, (int64_t)hk * d, 2) ||
            !slab_ok("dq_accum", seqlen_q, hd_bucket(d), 4) ||
            !bwd_rows_ok((int64_t)batch_size * seqlen_q, h, d)) return;
        const int64_t tok = (int64_t)batch_size * seqlen_q;
        int slices = bwd_slices(tok, batch_size, h, hk, d, seqlen_k, deterministic);
        char* ws = (char*)workspace;
        if (ws) {
            const int fit = bwd_slices_fit(tok, h, d, workspace_bytes);
            REQUIRE(fit >= 1, "workspace too small (%zu < %zu bytes)", workspace_bytes, bwd_ws_bytes(tok, h, d, 1));
            slices = std::min(slices, fit);
        }
        const size_t need = bwd_ws_bytes(tok, h, d, slices);
        if (!ws) ws = (char*)pool_get(stream, need);
        REQUIRE(ws, "could not allocate %zu bytes of backward scratch", need);
        const int hd = hd_bucket(d);
        BwdParams p{};
        p.q = q; p.k = k; p.v = v; p.o = out; p.dout = dout; p.lse = (const float*)softmax_lse;
        p.dq = dq; p.dk = dk; p.dv = dv;
        p.dq_accum = (float*)ws;
        const size_t acc = bwd_acc_bytes((int64_t)batch_size * seqlen_q, h, d);
        p.dsum = softmax_d ? (float*)softmax_d : (float*)(ws + slices * acc);
        p.lse_fix = (float*)(ws + slices * acc + bwd_dsum_bytes((int64_t)batch_size * seqlen_q, h));
        p.dq_slices = deterministic ? slices : 0;   // slices a workgroup walks into
        p.acc_slice = (int64_t)(acc / sizeof(float));
        p.q_row = (int64_t)h * d; p.q_head = d; p.q_batch = (int64_t)seqlen_q * h * d;
        p.o_row = p.q_row; p.o_head = d; p.o_batch = p.q_batch;
        p.do_row = p.q_row; p.do_head = d; p.do_batch = p.q_batch;
        p.dq_row = p.q_row; p.dq_head = d; p.dq_batch = p.q_batch;
        p.k_row = (int64_t)hk * d; p.k_head = d; p.k_batch = (int64_t)seqlen_k * hk * d;
        p.v_row = p.k_row; p.v_head = d; p.v_batch = p.k_batch;
        p.dk_row = p.k_row; p.dk_head = d; p.dk_batch = p.k_batch;
        p.dv_row = p.k_row; p.dv_head = d; p.dv_batch = p.k_batch;
        p.lse_batch = (int64_t)h * seqlen_q; p.lse_head = seqlen_q;
        p.acc_row = hd; p.acc_head = (int64_t)seqlen_q * hd; p.acc_batch = (int64_t)h * seqlen_q * hd;
        p.alibi = (const float*)alibi_slopes;
        p.alibi_bstride = batch_size > 1 ? num_heads : 0;
        p.b = batch_size; p.h = h; p.hk = hk; p.group = h / hk; p.d = d;
        p.seqlen_q = seqlen_q; p.seqlen_k = seqlen_k;
        bwd_common(p, softmax_scale, softcap, window_size_left, window_size_right, seqlen_k);
        if (!set_dropout(p, p_dropout, softcap)) return;
        if (!bwd_lse_convention(p, stream)) return;
        hip_ok(dispatch_bwd(p, !is_fp16, stream), "backward launch");
    } catch (...) {
        fail(9, "internal error in fmha_bwd");
    }
}

void fmha_varlen_bwd(void* dout, void* q, void* k, void* v, void* out, void* softmax_lse,
                     void* dq, void* dk, void* dv, void* cu_seqlens_q, void* cu_seqlens_k,
                     void* alibi_slopes, int32_t alibi_batch_stride, int32_t max_seqlen_q,
                     int32_t max_seqlen_k, int32_t total_q, int32_t total_k,
                     int32_t batch_size, int32_t num_heads, int32_t num_heads_k,
                     int32_t head_size, float softmax_scale, int window_size_left,
                     int window_size_right, float softcap, bool deterministic, bool is_fp16,
                     hipStream_t stream, void* workspace, size_t workspace_bytes,
                     void* softmax_d, float p_dropout) {
    try {
        clear_error();
        DevRngScope rng_scope;
        if (!check_common(q, k, v, out, batch_size, num_heads, num_heads_k, head_size)) return;
        REQUIRE(head_size <= 256, "the backward supports head dimension at most 256 (got %d)", head_size);
        REQUIRE(dout && softmax_lse && dq && dk && dv, "dout/softmax_lse/dq/dk/dv must be non-null");
        REQUIRE(!(softcap > 0.f && p_dropout > 0.f), "Softcapping does not support dropout for now");
        REQUIRE(cu_seqlens_q && cu_seqlens_k, "cu_seqlens_q/cu_seqlens_k must be non-null");
        REQUIRE(total_q > 0 && total_k > 0 && max_seqlen_q > 0 && max_seqlen_k > 0,
                "total/max sequence lengths must be positive");
        const int h = num_heads, hk = num_heads_k, d = head_size;
        if (!slab_ok("q/out/dout/dq", max_seqlen_q, (int64_t)h * d, 2) ||
            !slab_ok("k/v/dk/dv", max_seqlen_k, (int64_t)hk * d, 2) ||
            !slab_ok("dq_accum", max_seqlen_q, hd_bucket(d), 4) ||
            !bwd_rows_ok(total_q, h, d)) return;
        int slices = bwd_slices(total_q, batch_size, h, hk, d, max_seqlen_k, deterministic);
        char* ws = (char*)workspace;
        if (ws) {
            const int fit = bwd_slices_fit(total_q, h, d, workspace_bytes);
            REQUIRE(fit >= 1, "workspace too small (%zu < %zu bytes)", workspace_bytes, bwd_ws_bytes(total_q, h, d, 1));
            slices = std::min(slices, fit);
        }
        const size_t need = bwd_ws_bytes(total_q, h, d, slices);
        if (!ws) ws = (char*)pool_get(stream, need);
        REQUIRE(ws, "could not allocate %zu bytes of backward scratch", need);
        const int hd = hd_bucket(d);
        BwdParams p{};
        p.q = q; p.k = k; p.v = v; p.o = out; p.dout = dout; p.lse = (const float*)softmax_lse;
        p.dq = dq; p.dk = dk; p.dv = dv;
        p.dq_accum = (float*)ws;
        const size_t acc = bwd_acc_bytes(total_q, h, d);
        p.dsum = softmax_d ? (float*)softmax_d : (float*)(ws + slices * acc);
        p.lse_fix = (float*)(ws + slices * acc + bwd_dsum_bytes(total_q, h));
        p.dq_slices = deterministic ? slices : 0;   // slices a workgroup walks into
        p.acc_slice = (int64_t)(acc / sizeof(float));
        p.q_row = (int64_t)h * d; p.q_head = d; p.q_batch = 0;
        p.o_row = p.q_row; p.o_head = d; p.o_batch = 0;
        p.do_row = p.q_row; p.do_head = d; p.do_batch = 0;
        p.dq_row = p.q_row; p.dq_head = d; p.dq_batch = 0;
        p.k_row = (int64_t)hk * d; p.k_head = d; p.k_batch = 0;
        p.v_row = p.k_row; p.v_head = d; p.v_batch = 0;
        p.dk_row = p.k_row; p.dk_head = d; p.dk_batch = 0;
        p.dv_row = p.k_row; p.dv_head = d; p.dv_batch = 0;
        p.lse_batch = 0; p.lse_head = total_q;                 // LSE [h, total_q]
        p.acc_row = hd; p.acc_head = (int64_t)total_q * hd; p.acc_batch = 0;
        p.cu_seqlens_q = (const int*)cu_seqlens_q;
        p.cu_seqlens_k = (const int*)cu_seqlens_k;
        p.alibi = (const float*)alibi_slopes;
        p.alibi_bstride = alibi_batch_stride;
        p.b = batch_size; p.h = h; p.hk = hk; p.group = h / hk; p.d = d;
        p.seqlen_q = max_seqlen_q; p.seqlen_k = max_seqlen_k;
        bwd_common(p, softmax_scale, softcap, window_size_left, window_size_right, max_seqlen_k);
        if (!set_dropout(p, p_dropout, softcap)) return;
        if (!bwd_lse_convention(p, stream)) return;
        hip_ok(dispatch_bwd(p, !is_fp16, stream), "varlen backward launch");
    } catch (...) {
        fail(9, "internal error in fmha_varlen_bwd");
    }
}

}  // extern "C"
