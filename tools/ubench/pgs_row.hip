// Microbenchmark (diagnostic, not shipped): cycles per Gauss-Seidel row of the physics kernel's PGS
// sweep (he_physics.hip pgs_sweep_fix) in isolation, one wave per workgroup, by form:
//   0 shipped: v_pk_fma (cd, hi) + v_fma (lo) + v_med3 + v_readlane + v_writelane (the row's change)
//   1 the same without the v_writelane (the change not recorded: timing only)
//   2 three plain v_fma instead of the packed pair + one
//   3 two independent sweeps interleaved (ILP 2): per row cost of each
//   4 the change kept by a v_cndmask of the clamped vector under a constant lane mask (2 s_mov + select)
//   5 the change kept by a v_cmp of the lane id + v_cndmask
//   6 ILP 2 without the v_writelane
//   7 the v_writelane of row R issued in row R+1's block (after its v_med3), rows fenced by sched_barrier
//   8 form 0 under s_setprio 3 (the kernel's PGS priority)
//   9 form 0 with every row's change through one SGPR pair s[6:7], as the kernel's allocator does
// Waves per SIMD from the grid: 1024 workgroups = 1 per SIMD, 2048 = 2 (the kernel's occupancy), 3072 = 3, 4096 = 4.
// Output: median cycles per row update over the waves (s_memtime around S sweeps of N rows).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <cstdint>

typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int N = 32, S = 64;

template <int LANE>
__device__ __forceinline__ float wrlane(float v, float old) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(old) : "s"(v), "i"(LANE));
    return old;
}
__device__ __forceinline__ float rdlane(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }

template <int R>
__device__ __forceinline__ void row7(f2v& ch, float& lo, float& dvec, float dprev, const f2v (&ak)[N]) {
    if constexpr (R < N) {
        const float m = __builtin_amdgcn_fmed3f(ch.x, lo, ch.y);
        if constexpr (R > 0) dvec = wrlane<R - 1>(dprev, dvec);
        const float d = rdlane(m, R);
        ch = __builtin_elementwise_fma(ak[R], f2v{d, d}, ch);
        lo = fmaf(-ak[R].y, d, lo);
        __builtin_amdgcn_sched_barrier(0);
        row7<R + 1>(ch, lo, dvec, d, ak);
    } else {
        dvec = wrlane<N - 1>(dprev, dvec);
    }
}
template <int V, int R>
__device__ __forceinline__ void row(f2v& ch, float& lo, float& dvec, const f2v (&ak)[N]) {
    if constexpr (R < N) {
        const float m = __builtin_amdgcn_fmed3f(ch.x, lo, ch.y);
        if constexpr (V == 4) {
            uint32_t a, b;
            asm volatile("s_mov_b32 %0, %1" : "=s"(a) : "i"((uint32_t)(1ull << R)));
            asm volatile("s_mov_b32 %0, %1" : "=s"(b) : "i"((uint32_t)((1ull << R) >> 32)));
            dvec = __builtin_amdgcn_inverse_ballot_w64(((uint64_t)b << 32) | a) ? m : dvec;
        }
        if constexpr (V == 5) dvec = (int)threadIdx.x == R ? m : dvec;
        const float d = rdlane(m, R);
        if constexpr (V == 2) {
            ch.x = fmaf(ak[R].x, d, ch.x);
            ch.y = fmaf(ak[R].y, d, ch.y);
        } else {
            ch = __builtin_elementwise_fma(ak[R], f2v{d, d}, ch);
        }
        lo = fmaf(-ak[R].y, d, lo);
        if constexpr (V == 0 || V == 2 || V == 8) dvec = wrlane<R>(d, dvec);
        row<V, R + 1>(ch, lo, dvec, ak);
    }
}
// form 9: the shipped row with every row's change through the same SGPR pair s[6:7] (as the kernel's
// allocator does), written as one asm block per row with the compiler's hazard nops
template <int R>
__device__ __forceinline__ void row9(f2v& ch, float& lo, float& dvec, const f2v (&ak)[N]) {
    if constexpr (R < N) {
        float m;
        asm volatile(
            "v_med3_f32 %[m], %[cx], %[lo], %[cy]\n"
            "s_nop 0\n"
            "v_readlane_b32 s6, %[m], %[r]\n"
            "v_writelane_b32 %[dv], s6, %[r]\n"
            "s_nop 1\n"
            "v_pk_fma_f32 %[ch], %[ak], s[6:7], %[ch] op_sel_hi:[1,0,1]\n"
            "v_fma_f32 %[lo], -%[aky], s6, %[lo]"
            : [m] "=&v"(m), [ch] "+v"(ch), [lo] "+v"(lo), [dv] "+v"(dvec)
            : [cx] "v"(ch.x), [cy] "v"(ch.y), [ak] "v"(ak[R]), [aky] "v"(ak[R].y), [r] "i"(R)
            : "s6", "s7");
        row9<R + 1>(ch, lo, dvec, ak);
    }
}
template <int R, bool WL>
__device__ __forceinline__ void row2(f2v& ch, float& lo, float& dvec, f2v& ch2, float& lo2, float& dvec2,
                                     const f2v (&ak)[N]) {
    if constexpr (R < N) {
        const float d = rdlane(__builtin_amdgcn_fmed3f(ch.x, lo, ch.y), R);
        const float e = rdlane(__builtin_amdgcn_fmed3f(ch2.x, lo2, ch2.y), R);
        ch = __builtin_elementwise_fma(ak[R], f2v{d, d}, ch);
        ch2 = __builtin_elementwise_fma(ak[R], f2v{e, e}, ch2);
        lo = fmaf(-ak[R].y, d, lo);
        lo2 = fmaf(-ak[R].y, e, lo2);
        if constexpr (WL) {
            dvec = wrlane<R>(d, dvec);
            dvec2 = wrlane<R>(e, dvec2);
        }
        row2<R + 1, WL>(ch, lo, dvec, ch2, lo2, dvec2, ak);
    }
}

template <int V>
__global__ void __launch_bounds__(64) k(const float* in, float* out, unsigned long long* cyc) {
    const int l = threadIdx.x;
    f2v ak[N];
#pragma unroll
    for (int r = 0; r < N; ++r) ak[r] = f2v{in[r * 64 + l] * -0.01f, in[(r + N) * 64 + l] * 0.001f};
    f2v ch = {in[l] * 0.1f, 1e30f}, ch2 = {in[64 + l] * 0.1f, 1e30f};
    float lo = -1.f, lo2 = -1.f, dv = 0.f, dv2 = 0.f;
    __builtin_amdgcn_s_waitcnt(0);
    if constexpr (V == 8) __builtin_amdgcn_s_setprio(3);  // form 8: form 0 under the kernel's PGS priority
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int s = 0; s < S; ++s) {
        if constexpr (V == 9) row9<0>(ch, lo, dv, ak);
        else if constexpr (V == 3) row2<0, true>(ch, lo, dv, ch2, lo2, dv2, ak);
        else if constexpr (V == 6) row2<0, false>(ch, lo, dv, ch2, lo2, dv2, ak);
        else if constexpr (V == 7) row7<0>(ch, lo, dv, 0.f, ak);
        else row<V, 0>(ch, lo, dv, ak);
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    out[blockIdx.x * 64 + l] = ch.x + ch.y + lo + dv + ch2.x + lo2 + dv2;
    if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
double run(int blocks, const float* din, float* dout, unsigned long long* dcyc) {
    k<V><<<blocks, 64>>>(din, dout, dcyc);
    hipDeviceSynchronize();
    k<V><<<blocks, 64>>>(din, dout, dcyc);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(blocks);
    hipMemcpy(c.data(), dcyc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    return (double)c[blocks / 2] / (S * N);
}

int main() {
    const int maxb = 4096;
    std::vector<float> h(2 * N * 64 + 256);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 1000.f;
    float *din, *dout;
    unsigned long long* dcyc;
    hipMalloc(&din, h.size() * 4);
    hipMalloc(&dout, maxb * 64 * 4);
    hipMalloc(&dcyc, maxb * 8);
    hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    for (int b : {1024, 2048, 3072, 4096}) {
        printf("{\"waves_per_simd\": %d, \"form0_shipped\": %.1f, \"form1_no_writelane\": %.1f, \"form2_plain_fma\": %.1f, "
               "\"form3_ilp2_per_row\": %.1f, \"form4_mask_select\": %.1f, \"form5_cmp_select\": %.1f, "
               "\"form6_ilp2_no_writelane\": %.1f, \"form7_deferred_writelane\": %.1f, \"form8_setprio3\": %.1f, "
               "\"form9_one_sgpr_pair\": %.1f}\n", b / 1024, run<0>(b, din, dout, dcyc), run<1>(b, din, dout, dcyc),
               run<2>(b, din, dout, dcyc), run<3>(b, din, dout, dcyc) / 2.0, run<4>(b, din, dout, dcyc),
               run<5>(b, din, dout, dcyc), run<6>(b, din, dout, dcyc) / 2.0, run<7>(b, din, dout, dcyc),
               run<8>(b, din, dout, dcyc), run<9>(b, din, dout, dcyc));
    }
    return 0;
}
