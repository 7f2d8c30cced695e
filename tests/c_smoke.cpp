// c_smoke.cpp — a torch-free C++ caller of libpaged-attention.so (the analogue of the
// reference's test.cc:10-80, which hipMallocs buffers and calls fmha_fwd from plain C++).
//
// It reads one golden case dumped as raw little-endian files (tests/test_c_smoke_gpu.py writes
// them from a committed fixture): q, k, v, dout [b, s, h, d] in fp16/bf16, the oracle's
// out_ref / dq_ref / dk_ref / dv_ref (fp32), and the pass bounds.  It then calls, through the
// C ABI only,
//   fmha_fwd                the dense forward (also writes the LSE),
//   fmha_varlen_fwd         the same batch packed as cu_seqlens sequences,
//   fmha_page_kvcache_fwd   the same K/V copied into a paged cache (page 16, reversed page
//                           order in the block table),
//   fmha_bwd                dq, dk, dv from dout and the forward's O / LSE,
// copies the results back and checks max |x - ref| <= bound for each; prints one line per
// check and "C_SMOKE_OK" when all pass (exit status 0), else exits 1.
//
//   c_smoke <dir>   (dir holds meta.txt and the .bin files)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "paged_attn.h"

#define HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(2); } } while (0)

static std::vector<char> read_file(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { std::fprintf(stderr, "cannot open %s\n", path.c_str()); std::exit(2); }
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<char> buf(n);
    if (n && std::fread(buf.data(), 1, n, f) != (size_t)n) { std::fprintf(stderr, "short read %s\n", path.c_str()); std::exit(2); }
    std::fclose(f);
    return buf;
}

static float half_to_f32(uint16_t h) {
    const uint32_t s = (uint32_t)(h & 0x8000) << 16, e = (h >> 10) & 0x1F, m = h & 0x3FF;
    uint32_t bits;
    if (e == 0) {
        if (m == 0) bits = s;
        else {   // subnormal
            float f = std::ldexp((float)m, -24);
            return s ? -f : f;
        }
    } else if (e == 31) bits = s | 0x7F800000u | (m << 13);
    else bits = s | ((e + 112) << 23) | (m << 13);
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}
static float bf16_to_f32(uint16_t h) {
    const uint32_t bits = (uint32_t)h << 16;
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

struct Case {
    int b, h, hk, sq, sk, d, causal, fp16;
    float scale, fwd_bound, dq_bound, dk_bound, dv_bound;
};

static float max_err(const std::vector<uint16_t>& x, const std::vector<float>& ref, bool fp16) {
    float m = 0.f;
    for (size_t i = 0; i < x.size(); ++i) {
        const float v = fp16 ? half_to_f32(x[i]) : bf16_to_f32(x[i]);
        const float e = std::fabs(v - ref[i]);
        if (!(e <= m)) m = (e != e) ? INFINITY : e;
    }
    return m;
}

template <typename T>
static T* dev_from(const std::vector<char>& host) {
    T* p = nullptr;
    HIP(hipMalloc(&p, host.size() ? host.size() : 16));
    if (host.size()) HIP(hipMemcpy(p, host.data(), host.size(), hipMemcpyHostToDevice));
    return p;
}

static std::vector<uint16_t> to_host16(const void* dev, size_t n) {
    std::vector<uint16_t> h(n);
    HIP(hipMemcpy(h.data(), dev, n * 2, hipMemcpyDeviceToHost));
    return h;
}

static std::vector<float> as_f32(const std::vector<char>& b) {
    std::vector<float> f(b.size() / 4);
    std::memcpy(f.data(), b.data(), b.size());
    return f;
}

int main(int argc, char** argv) {
    if (argc != 2) { std::fprintf(stderr, "usage: c_smoke <dir>\n"); return 2; }
    const std::string dir = argv[1];
    Case c{};
    {
        FILE* f = std::fopen((dir + "/meta.txt").c_str(), "r");
        if (!f || std::fscanf(f, "%d %d %d %d %d %d %d %d %f %f %f %f %f", &c.b, &c.h, &c.hk, &c.sq, &c.sk,
                              &c.d, &c.causal, &c.fp16, &c.scale, &c.fwd_bound, &c.dq_bound, &c.dk_bound,
                              &c.dv_bound) != 13) {
            std::fprintf(stderr, "bad meta.txt\n");
            return 2;
        }
        std::fclose(f);
    }
    std::printf("case b=%d h=%d hk=%d sq=%d sk=%d d=%d causal=%d %s  library %s\n", c.b, c.h, c.hk, c.sq,
                c.sk, c.d, c.causal, c.fp16 ? "fp16" : "bf16", fmha_version());
    const auto hq = read_file(dir + "/q.bin"), hkk = read_file(dir + "/k.bin"), hv = read_file(dir + "/v.bin");
    const auto hdo = read_file(dir + "/dout.bin");
    const auto out_ref = as_f32(read_file(dir + "/out_ref.bin"));
    const auto dq_ref = as_f32(read_file(dir + "/dq_ref.bin"));
    const auto dk_ref = as_f32(read_file(dir + "/dk_ref.bin"));
    const auto dv_ref = as_f32(read_file(dir + "/dv_ref.bin"));
    const size_t nq = (size_t)c.b * c.sq * c.h * c.d, nk = (size_t)c.b * c.sk * c.hk * c.d;
    if (hq.size() != nq * 2 || hkk.size() != nk * 2 || hv.size() != nk * 2 || out_ref.size() != nq) {
        std::fprintf(stderr, "size mismatch\n");
        return 2;
    }
    void *q = dev_from<char>(hq), *k = dev_from<char>(hkk), *v = dev_from<char>(hv), *dout = dev_from<char>(hdo);
    void *o, *o2, *o3, *dq, *dk, *dv;
    float* lse;
    HIP(hipMalloc(&o, nq * 2)); HIP(hipMalloc(&o2, nq * 2)); HIP(hipMalloc(&o3, nq * 2));
    HIP(hipMalloc(&dq, nq * 2)); HIP(hipMalloc(&dk, nk * 2)); HIP(hipMalloc(&dv, nk * 2));
    HIP(hipMalloc(&lse, (size_t)c.b * c.h * c.sq * 4));
    hipStream_t st;
    HIP(hipStreamCreate(&st));
    const int wl = -1, wr = c.causal ? 0 : -1;
    bool ok = true;
    auto report = [&](const char* what, float err, float bound) {
        const bool pass = err <= bound;
        ok = ok && pass;
        std::printf("%-24s max|err| %.3e  bound %.3e  %s\n", what, err, bound, pass ? "ok" : "FAIL");
    };
    auto api_ok = [&](const char* what) {
        if (fmha_last_status() != 0) {
            std::printf("%s: error: %s\n", what, fmha_last_error());
            ok = false;
            return false;
        }
        return true;
    };

    // 1) fmha_fwd (the reference's signature, csrc/paged_attn.h:8-31)
    fmha_fwd(q, k, v, o, nullptr, c.sq, c.sk, c.b, c.h, c.hk, c.d, 0.f, st, nullptr, c.scale, nullptr, lse,
             wl, wr, 0.f, false, c.fp16 != 0, 0);
    if (api_ok("fmha_fwd")) {
        HIP(hipStreamSynchronize(st));
        report("fmha_fwd", max_err(to_host16(o, nq), out_ref, c.fp16), c.fwd_bound);
    }

    // 2) fmha_varlen_fwd: the batch as packed sequences (csrc/paged_attn.h:33-53)
    {
        std::vector<int> cq(c.b + 1), ck(c.b + 1);
        for (int i = 0; i <= c.b; ++i) { cq[i] = i * c.sq; ck[i] = i * c.sk; }
        int *dcq, *dck;
        HIP(hipMalloc(&dcq, cq.size() * 4)); HIP(hipMalloc(&dck, ck.size() * 4));
        HIP(hipMemcpy(dcq, cq.data(), cq.size() * 4, hipMemcpyHostToDevice));
        HIP(hipMemcpy(dck, ck.data(), ck.size() * 4, hipMemcpyHostToDevice));
        fmha_varlen_fwd(q, k, v, o2, dcq, dck, c.sq, c.sk, c.b, c.h, c.hk, c.d, st, c.scale, c.causal != 0,
                        c.fp16 != 0, wl, wr);
        if (api_ok("fmha_varlen_fwd")) {
            HIP(hipStreamSynchronize(st));
            report("fmha_varlen_fwd", max_err(to_host16(o2, nq), out_ref, c.fp16), c.fwd_bound);
        }
        HIP(hipFree(dcq)); HIP(hipFree(dck));
    }

    // 3) fmha_page_kvcache_fwd: K/V copied into pages of 16 rows, pages in reversed order
    //    (csrc/paged_attn.h:55-84; block_table stride = max_cache_seq_k / page)
    {
        const int page = 16, per_seq = (c.sk + page - 1) / page, nblocks = c.b * per_seq;
        const size_t row = (size_t)c.hk * c.d * 2;       // bytes of one cache row
        std::vector<char> kc((size_t)nblocks * page * row, 0), vc(kc.size(), 0);
        std::vector<int> table(nblocks), seqlens(c.b, c.sk);
        for (int bi = 0; bi < c.b; ++bi)
            for (int pi = 0; pi < per_seq; ++pi) {
                const int blk = nblocks - 1 - (bi * per_seq + pi);
                table[bi * per_seq + pi] = blk;
                for (int r = 0; r < page; ++r) {
                    const int s = pi * page + r;
                    if (s >= c.sk) break;
                    std::memcpy(&kc[((size_t)blk * page + r) * row], &hkk[((size_t)bi * c.sk + s) * row], row);
                    std::memcpy(&vc[((size_t)blk * page + r) * row], &hv[((size_t)bi * c.sk + s) * row], row);
                }
            }
        void *dkc = dev_from<char>(kc), *dvc = dev_from<char>(vc);
        std::vector<char> tb((char*)table.data(), (char*)table.data() + table.size() * 4);
        std::vector<char> sl((char*)seqlens.data(), (char*)seqlens.data() + seqlens.size() * 4);
        void *dtb = dev_from<char>(tb), *dsl = dev_from<char>(sl);
        fmha_page_kvcache_fwd(q, dkc, dvc, nullptr, nullptr, o3, dtb, dsl, per_seq * page, c.sq, c.sk, c.b,
                              c.h, c.hk, c.d, page, st, c.scale, wl, wr, 0, nullptr, nullptr, nullptr,
                              c.causal != 0, false, c.fp16 != 0);
        if (api_ok("fmha_page_kvcache_fwd")) {
            HIP(hipStreamSynchronize(st));
            report("fmha_page_kvcache_fwd", max_err(to_host16(o3, nq), out_ref, c.fp16), c.fwd_bound);
        }
        HIP(hipFree(dkc)); HIP(hipFree(dvc)); HIP(hipFree(dtb)); HIP(hipFree(dsl));
    }

    // 4) fmha_bwd (a new symbol: the reference never built mha_bwd) from the forward's O / LSE
    fmha_bwd(dout, q, k, v, o, lse, dq, dk, dv, nullptr, nullptr, c.sq, c.sk, c.b, c.h, c.hk, c.d, 0.f,
             c.scale, wl, wr, 0.f, false, c.fp16 != 0, st, nullptr, 0);
    if (api_ok("fmha_bwd")) {
        HIP(hipStreamSynchronize(st));
        report("fmha_bwd dq", max_err(to_host16(dq, nq), dq_ref, c.fp16), c.dq_bound);
        report("fmha_bwd dk", max_err(to_host16(dk, nk), dk_ref, c.fp16), c.dk_bound);
        report("fmha_bwd dv", max_err(to_host16(dv, nk), dv_ref, c.fp16), c.dv_bound);
    }

    for (void* p : {q, k, v, dout, o, o2, o3, dq, dk, dv}) HIP(hipFree(p));
    HIP(hipFree(lse));
    HIP(hipStreamDestroy(st));
    std::printf(ok ? "C_SMOKE_OK\n" : "C_SMOKE_FAIL\n");
    return ok ? 0 : 1;
}
