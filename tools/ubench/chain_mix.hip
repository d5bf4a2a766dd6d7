// Microbenchmark (diagnostic, not shipped): how waves that are latency-bound on their own share a
// SIMD, as a proxy for the physics kernel at 1-4 waves per SIMD (DESIGN §10 occupancy plan). One
// wave per workgroup runs S iterations of a dependent chain shaped like the kernel's serial phases
// (an LDS store, the in-order LDS broadcast read behind it, three dependent FMAs, a v_readlane into
// an SGPR that the next iteration's FMA reads) plus F independent FMAs per iteration on other
// registers (the ILP the compiler finds beside the chain). Waves per SIMD from the grid: 1024
// workgroups = 1 per SIMD ... 4096 = 4. Output: median cycles per iteration, and per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

constexpr int S = 256;

template <int F>
__global__ void __launch_bounds__(64) k(const float* in, float* out, unsigned long long* cyc) {
    __shared__ float lds[64];
    const int l = threadIdx.x;
    float x = in[l], acc[F > 0 ? F : 1];
#pragma unroll
    for (int j = 0; j < (F > 0 ? F : 1); ++j) acc[j] = in[64 + j] + l;
    const float a = in[200], b = in[201];
    lds[l] = x;
    __builtin_amdgcn_wave_barrier();
    const unsigned long long t0 = __builtin_readcyclecounter();
#pragma unroll 1
    for (int s = 0; s < S; ++s) {
        float t = lds[(s * 7) & 63];  // broadcast read behind the previous iteration's store
        t = fmaf(t, a, b);
        t = fmaf(t, a, x);
        t = fmaf(t, b, a);
        const float u = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(t), s & 63));
#pragma unroll
        for (int j = 0; j < F; ++j) acc[j] = fmaf(acc[j], a, u * (j + 1));
        x = fmaf(x, u, t);
        lds[l] = x;
        __builtin_amdgcn_wave_barrier();
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    float r = x;
#pragma unroll
    for (int j = 0; j < F; ++j) r += acc[j];
    out[blockIdx.x * 64 + l] = r;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int F>
double run(int blocks, const float* din, float* dout, unsigned long long* dcyc) {
    k<F><<<blocks, 64>>>(din, dout, dcyc);
    hipDeviceSynchronize();
    k<F><<<blocks, 64>>>(din, dout, dcyc);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(blocks);
    hipMemcpy(c.data(), dcyc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    return (double)c[blocks / 2] / S;
}

int main() {
    const int maxb = 4096;
    std::vector<float> h(256);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 0.5f + (float)((i * 2654435761u) % 1000) / 4000.f;
    h[200] = 0.999f;
    h[201] = 0.001f;
    float *din, *dout;
    unsigned long long* dcyc;
    hipMalloc(&din, h.size() * 4);
    hipMalloc(&dout, maxb * 64 * 4);
    hipMalloc(&dcyc, maxb * 8);
    hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    for (int b : {1024, 2048, 3072, 4096})
        printf("{\"waves_per_simd\": %d, \"cycles_per_iter\": {\"F0\": %.1f, \"F4\": %.1f, \"F8\": %.1f, \"F16\": %.1f, \"F24\": %.1f, \"F32\": %.1f}}\n",
               b / 1024, run<0>(b, din, dout, dcyc), run<4>(b, din, dout, dcyc), run<8>(b, din, dout, dcyc),
               run<16>(b, din, dout, dcyc), run<24>(b, din, dout, dcyc), run<32>(b, din, dout, dcyc));
    return 0;
}
