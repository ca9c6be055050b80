// Checks the DPP register-transpose line FFT against the LDS-exchange one (must be bit-identical)
// for both transform directions, for each GD_DPP_ROR_DIR build.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DGD_DPP_ROR_DIR=-1] -o tools/dpp_check tools/dpp_check.hip
#include "../galaxy-deconv_amd/csrc/gd_fft.hpp"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace gd;

template <bool INV, bool DPP>
__global__ __launch_bounds__(256) void k_fft_check(const float2* in, float2* out) {
    __shared__ float2 tw[256];
    __shared__ float2 xch[16 * xch_elems<256>()];
    const int tid = threadIdx.x, line = tid / 16, j = tid % 16;
    fill_twiddles<256>(tw, tid, 256);
    __syncthreads();
    float2 v[16];
    const float2* src = in + (blockIdx.x * 16 + line) * 256;
    for (int r = 0; r < 16; ++r) v[r] = src[j + 16 * r];
    line_fft<256, INV, false, DPP>(v, j, xch + line * xch_elems<256>(), tw);
    float2* dst = out + (blockIdx.x * 16 + line) * 256;
    for (int r = 0; r < 16; ++r) dst[j + 16 * r] = v[r];
}

int main() {
    const int lines = 64 * 16, n = lines * 256;
    std::vector<float2> h(n);
    srand(7);
    for (auto& x : h) x = make_float2(rand() / float(RAND_MAX) - 0.5f, rand() / float(RAND_MAX) - 0.5f);
    float2 *in, *o1, *o2;
    hipMalloc(&in, n * 8); hipMalloc(&o1, n * 8); hipMalloc(&o2, n * 8);
    hipMemcpy(in, h.data(), n * 8, hipMemcpyHostToDevice);
    std::vector<float2> a(n), b(n);
    for (int inv = 0; inv < 2; ++inv) {
        if (inv) {
            hipLaunchKernelGGL((k_fft_check<true, false>), dim3(64), dim3(256), 0, 0, in, o1);
            hipLaunchKernelGGL((k_fft_check<true, true>), dim3(64), dim3(256), 0, 0, in, o2);
        } else {
            hipLaunchKernelGGL((k_fft_check<false, false>), dim3(64), dim3(256), 0, 0, in, o1);
            hipLaunchKernelGGL((k_fft_check<false, true>), dim3(64), dim3(256), 0, 0, in, o2);
        }
        if (hipDeviceSynchronize() != hipSuccess) { printf("HIP error\n"); return 1; }
        hipMemcpy(a.data(), o1, n * 8, hipMemcpyDeviceToHost);
        hipMemcpy(b.data(), o2, n * 8, hipMemcpyDeviceToHost);
        int bad = 0;
        double md = 0;
        for (int i = 0; i < n; ++i) {
            if (a[i].x != b[i].x || a[i].y != b[i].y) ++bad;
            md = fmax(md, fabs(a[i].x - b[i].x) + fabs(a[i].y - b[i].y));
        }
        printf("dir %d inv %d: %d of %d values differ, max |diff| %.3e\n", GD_DPP_ROR_DIR, inv, bad, n, md);
    }
    return 0;
}
