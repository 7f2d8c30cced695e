// The dQ-atomic floor of the C3 backward, measured.
//
// The backward's main kernel adds every key block's dQ tile into the fp32 accumulator with float
// atomics (csrc/fmha_bwd_kernel.h; the reference does the same, flash_bwd_kernel_hip.h:637).
// This probe issues exactly that stream with nothing else: one workgroup of 512 threads per
// (batch x head, 256-key block), sweeping the 32-row query tiles its keys see under causal
// masking (tiles >= 8 kb), adding a 32 x 128 fp32 tile per step - 2.28 GB of atomic adds at the
// C3 shape (B4 H32 S4096 D128).  Its time is the floor under any backward that keeps the atomic
// dQ at 256 keys per workgroup.  Modes: 0 = atomic adds (no return), 1 = plain stores of the
// same bytes (the write-bandwidth reference), 2 = atomics in the order key block by key block
// (grid y outermost), 3-5 atomics XCD-local / sc1 / nt, 6 = the deterministic mode's stream
// (round 6): S = 2 single-writer slices, workgroup (bh, s) walking key
// blocks s, s + S, ... in snake order and adding by plain read-modify-write.
//
//   hipcc -O3 --offload-arch=gfx950 -munsafe-fp-atomics tools/probe/atomic_floor.hip -o tools/probe/atomic_floor
//   tools/probe/atomic_floor [iters]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int B = 4, H = 32, S = 4096, D = 128, KB = 256, QT = 32;

constexpr int NSLICE = 2;   // ceil(256 CUs / (B * H)) for C3

__global__ void __launch_bounds__(512) dq_rmw(float* acc) {
    const int bh = blockIdx.x, s = blockIdx.y, t = threadIdx.x;
    const int b = bh / H, h = bh % H;
    float* slice = acc + (size_t)s * B * S * H * D;
    for (int r = 0;; ++r) {
        const int kb = r * NSLICE + ((r & 1) ? NSLICE - 1 - s : s);
        if (kb >= S / KB) break;
        for (int qt = kb * (KB / QT); qt < S / QT; ++qt) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int e = i * 512 + t;
                const int row = qt * QT + e / D, col = e % D;
                float* p = slice + (((int64_t)b * S + row) * H + h) * D + col;
                *p = (r == 0 ? 0.f : *p) + 1e-3f * (float)(col + 1);   // first block writes
            }
        }
    }
}

// the same stream with the next tile's loads issued before this tile's stores (one tile of
// lookahead per thread, 16 loads in flight)
__global__ void __launch_bounds__(512) dq_rmw2(float* acc) {
    const int bh = blockIdx.x, s = blockIdx.y, t = threadIdx.x;
    const int b = bh / H, h = bh % H;
    float* slice = acc + (size_t)s * B * S * H * D;
    for (int r = 0;; ++r) {
        const int kb = r * NSLICE + ((r & 1) ? NSLICE - 1 - s : s);
        if (kb >= S / KB) break;
        const int q0 = kb * (KB / QT), q1 = S / QT;
        float cur[8], nxt[8];
        auto addr = [&](int qt, int i) {
            const int e = i * 512 + t;
            return slice + (((int64_t)b * S + qt * QT + e / D) * H + h) * D + e % D;
        };
#pragma unroll
        for (int i = 0; i < 8; ++i) cur[i] = r ? *addr(q0, i) : 0.f;
        for (int qt = q0; qt < q1; ++qt) {
            if (qt + 1 < q1) {
#pragma unroll
                for (int i = 0; i < 8; ++i) nxt[i] = r ? *addr(qt + 1, i) : 0.f;
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) *addr(qt, i) = cur[i] + 1e-3f * (float)((i * 512 + t) % D + 1);
#pragma unroll
            for (int i = 0; i < 8; ++i) cur[i] = nxt[i];
        }
    }
}

template <int MODE>
__global__ void __launch_bounds__(512) dq_stream(float* acc) {
    int bh = MODE == 2 ? blockIdx.y : blockIdx.x, kb = MODE == 2 ? blockIdx.x : blockIdx.y;
    if constexpr (MODE >= 3) {
        // 1-D grid, workgroup i on XCD i % 8 (round-robin dispatch): every key block of a
        // (b, h) on the XCD of bh % 8, so each dQ address is added to from one XCD only
        const int i = blockIdx.x;
        bh = (i / 128) * 8 + i % 8;
        kb = (i / 8) % 16;
    }
    const int t = threadIdx.x;
    const int b = bh / H, h = bh % H;
    // a 32 x 128 tile = 4096 floats: thread t adds 8, lanes of a wave 256 B apart per row pair
    for (int qt = kb * (KB / QT); qt < S / QT; ++qt) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int e = i * 512 + t;                   // element of the tile
            const int row = qt * QT + e / D, col = e % D;
            float* p = acc + (((int64_t)b * S + row) * H + h) * D + col;   // [B, S, H, D]
            const float v = 1e-3f * (float)(col + 1);
            if constexpr (MODE == 1) *p = v;
            else if constexpr (MODE == 4)       // the same add with the device-scope bit
                asm volatile("global_atomic_add_f32 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
            else if constexpr (MODE == 5)       // non-temporal
                asm volatile("global_atomic_add_f32 %0, %1, off nt" :: "v"(p), "v"(v) : "memory");
            else unsafeAtomicAdd(p, v);
        }
    }
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 10;
    const size_t n = (size_t)B * S * H * D;
    float* acc;
    if (hipMalloc(&acc, n * 4 * NSLICE) != hipSuccess) return 1;
    hipMemset(acc, 0, n * 4 * NSLICE);
    double bytes = 0;
    for (int kb = 0; kb < S / KB; ++kb) bytes += (double)(S / QT - kb * (KB / QT)) * QT * D * 4;
    bytes *= B * H;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[8] = {"atomic add (grid bh x kb)", "plain store (same bytes)", "atomic add (grid kb x bh)",
                            "atomic add (bh XCD-local)", "atomic add sc1 (XCD-local)", "atomic add nt (XCD-local)",
                            "RMW, 2 single-writer slices", "RMW, next tile's loads first"};
    for (int mode = 0; mode < 8; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {             // rep 0: warm-up
            hipEventRecord(e0);
            for (int it = 0; it < iters; ++it) {
                if (mode == 0) hipLaunchKernelGGL(dq_stream<0>, dim3(B * H, S / KB), dim3(512), 0, 0, acc);
                else if (mode == 1) hipLaunchKernelGGL(dq_stream<1>, dim3(B * H, S / KB), dim3(512), 0, 0, acc);
                else if (mode == 2) hipLaunchKernelGGL(dq_stream<2>, dim3(S / KB, B * H), dim3(512), 0, 0, acc);
                else if (mode == 3) hipLaunchKernelGGL(dq_stream<3>, dim3(B * H * S / KB), dim3(512), 0, 0, acc);
                else if (mode == 4) hipLaunchKernelGGL(dq_stream<4>, dim3(B * H * S / KB), dim3(512), 0, 0, acc);
                else if (mode == 5) hipLaunchKernelGGL(dq_stream<5>, dim3(B * H * S / KB), dim3(512), 0, 0, acc);
                else if (mode == 6) hipLaunchKernelGGL(dq_rmw, dim3(B * H, NSLICE), dim3(512), 0, 0, acc);
                else hipLaunchKernelGGL(dq_rmw2, dim3(B * H, NSLICE), dim3(512), 0, 0, acc);
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep) printf("%-28s %.3f ms per launch, %.3f GB, %.3f TB/s\n", names[mode], ms / iters,
                            bytes / 1e9, bytes / (ms / iters * 1e-3) / 1e12);
        }
    }
    // the sums of every mode must agree: check one element of the first row against mode 0
    if (hipGetLastError() != hipSuccess) return 2;
    hipFree(acc);
    return 0;
}
