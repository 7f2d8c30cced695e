// Layout probes for the fp8 forward (run once on an MI355X; results recorded in DESIGN.md):
//  1. ds_read_b64_tr_b8: what each lane of a wave receives, given per-lane row addresses into
//     an LDS byte image whose byte at (row, col) is row * 16 + col (rows of 16 bytes).
//  2. v_mfma_scale_f32_32x32x64_f8f6f4 (fp8 e4m3 A and B, E8M0 scales 127 = 1.0): which
//     (lane half, byte) slots of A and B are contracted together, checked with one-hot operands.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probe_fp8.hip -o tools/probe_fp8
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(2))) int i32x2;

__global__ void probe_tr_b8(unsigned char* out, int mode) {
    __shared__ unsigned char img[64 * 16];
    const int lane = threadIdx.x;
    for (int i = lane; i < 64 * 16; i += 64) img[i] = (unsigned char)(((i / 16) & 15) * 16 + (i % 16));
    __syncthreads();
    // mode 0: lane supplies the address of row (lane % 16) column 0 of block (lane / 16) * 16 rows
    // mode 1: lane 8q+p of each 16-lane group supplies row q (0..7 within block) column 8*(p&1)
    int addr;
    if (mode == 0) addr = (lane % 16) * 16;
    else {
        const int g = lane >> 4, i = lane & 15, q = i >> 1, pp = i & 1;
        addr = (g * 8 + q) * 16 + 8 * pp;
    }
    typedef __attribute__((address_space(3))) i32x2 lds_i32x2;
    const i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_i32x2*)((__attribute__((address_space(3))) char*)img + addr));
    const unsigned char* b = (const unsigned char*)&v;
    for (int e = 0; e < 8; ++e) out[lane * 8 + e] = b[e];
}

// fp8 e4m3fn 1.0 = 0x38
__global__ void probe_mfma(float* out, int ha, int ea, int hb, int eb) {
    const int lane = threadIdx.x;
    const int h = lane >> 5;
    i32x8 a = {}, b = {};
    unsigned char* pa = (unsigned char*)&a;
    unsigned char* pb = (unsigned char*)&b;
    if (h == ha) pa[ea] = 0x38;
    if (h == hb) pb[eb] = 0x38;
    f32x16 c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += c[r];
    out[lane] = s;
}

int main(int argc, char**) {
    unsigned char* d;
    hipMalloc(&d, 64 * 8);
    unsigned char h[64 * 8];
    for (int mode = 0; mode < 2; ++mode) {  // rows printed mod 16
        hipLaunchKernelGGL(probe_tr_b8, dim3(1), dim3(64), 0, 0, d, mode);
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        printf("tr_b8 mode %d (row,col) per lane:\n", mode);
        for (int l = 0; l < 64; ++l) {
            printf(" L%02d:", l);
            for (int e = 0; e < 8; ++e) printf(" %d,%d", h[l * 8 + e] / 16, h[l * 8 + e] % 16);
            printf("\n");
        }
    }
    if (argc > 1) return 0;   // tr_b8 only
    float* f;
    hipMalloc(&f, 64 * 4);
    float hf[64];
    // slot (ha, ea) of A against slot (hb, eb) of B: total over the 32x32 output
    int same = 0, cross = 0;
    for (int ha = 0; ha < 2; ++ha)
        for (int ea = 0; ea < 32; ++ea)
            for (int hb = 0; hb < 2; ++hb)
                for (int eb = 0; eb < 32; ++eb) {
                    hipLaunchKernelGGL(probe_mfma, dim3(1), dim3(64), 0, 0, f, ha, ea, hb, eb);
                    hipMemcpy(hf, f, sizeof(hf), hipMemcpyDeviceToHost);
                    float t = 0.f;
                    for (int l = 0; l < 64; ++l) t += hf[l];
                    if (t != 0.f) {
                        if (ha == hb && ea == eb) ++same;
                        else { ++cross; printf("cross: A(%d,%d) x B(%d,%d) = %g\n", ha, ea, hb, eb, t); }
                    }
                }
    printf("mfma scale 32x32x64: matching slots %d / 64, cross pairs %d\n", same, cross);
    return 0;
}
