// he_regla.h -- wave-resident dense linear algebra on the static SMPL dof tree (gfx950).
//
// The 75x75 joint-space inertia H lives in VGPRs, one column per lane: lane j holds c[i] =
// H[i][j] for every row i (entries with i >= j are the lower triangle; i < j slots are scratch),
// and lanes 0..10 additionally hold c2[i-64] = H[i][64+j] for the 11 dofs >= 64. Every loop over
// the tree is unrolled at compile time by template recursion over the constexpr tables in
// he_smpl_topo.h, so all register indices are immediates and the uniform factors travel through
// v_readlane -> SGPR. Branch-induced sparsity (RBDA 6.5) means no fill-in: entries outside a
// row's ancestor chain stay exactly zero.
#pragma once
#include <hip/hip_runtime.h>

#include "he_smpl_topo.h"

namespace regla {

using namespace smpl;
constexpr int W = 64;
constexpr int NG = kNG;
constexpr int NH = NG - 64;  // columns held in the second register set

struct RegMat {
    float c[NG];
    float c2[NH];
};

__device__ __forceinline__ float rdlane(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// v_writelane: `v` on lane `l` only
template <int LANE>
__device__ __forceinline__ float wrlane(float v, float old) {
    asm("v_writelane_b32 %0, %1, %2" : "+v"(old) : "s"(v), "i"(LANE));
    return old;
}

// H[ROW][COL] (ROW >= COL) from the owning lane, as a wave-uniform value
template <int ROW, int COL>
__device__ __forceinline__ float get(const RegMat& M) {
    static_assert(ROW >= COL, "lower triangle only");
    if constexpr (COL < 64) return rdlane(M.c[ROW], COL);
    else return rdlane(M.c2[ROW - 64], COL - 64);
}

// lanes whose bit is set in the compile-time mask C (v_cndmask on an SGPR-pair constant; no
// per-lane compare or branch)
template <uint64_t C>
__device__ __forceinline__ bool lanes() {
    // the constant is materialised here by two s_mov_b32 (volatile: never hoisted out of the
    // substep loop, where dozens of distinct masks would otherwise be kept live and spilled)
    uint32_t lo, hi;
    asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"((uint32_t)C));
    asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"((uint32_t)(C >> 32)));
    return __builtin_amdgcn_inverse_ballot_w64(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, W);
    return v;
}

// ---------------------------------------------------------------- LTDL factorisation
__device__ __forceinline__ float uniform(float v) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

// H[I][j] -= H[K][I] * L[K][j] for every column j (c[K] already scaled to row K of L)
template <int K, int X, int D>
__device__ __forceinline__ void fac_anc(RegMat& M, const float (&hk)[kMaxChain]) {
    if constexpr (X < D) {
        constexpr int I = kChain[K][X];
        M.c[I] -= hk[X] * M.c[K];
        if constexpr (I >= 64) M.c2[I - 64] -= hk[X] * M.c2[K - 64];
        fac_anc<K, X + 1, D>(M, hk);
    }
}
template <int K, int X, int D>
__device__ __forceinline__ void read_row(const RegMat& M, float (&hk)[kMaxChain]) {
    if constexpr (X < D) {
        hk[X] = get<K, kChain[K][X]>(M);
        read_row<K, X + 1, D>(M, hk);
    }
}

// elimination step S eliminates dof kElimOrder[S] (deepest first, so consecutive steps mostly lie
// on independent branches and can overlap; a scheduling barrier every two steps bounds the live
// SGPR/VGPR ranges). The pivot D_K is kept on its owning lane (Dl / D2); the pivot reciprocal and
// the row entries H[K][I] are wave-uniform (SGPRs), so each update is one FMA.
template <int S>
__device__ __forceinline__ void factor_steps(RegMat& M, float& Dl, float& D2) {
    if constexpr (S < NG) {
        constexpr int K = kElimOrder[S];
        constexpr int D = kDofNanc[K] - 1;
        const float dk = get<K, K>(M);
        const float inv = uniform(__builtin_amdgcn_rcpf(dk));  // v_rcp_f32 (1 ulp): short pivot chain
        float hk[kMaxChain];
        read_row<K, 0, D>(M, hk);
        M.c[K] *= inv;  // row K -> L[K][.] on lanes j < K
        if constexpr (K >= 64) M.c2[K - 64] *= inv;
        fac_anc<K, 0, D>(M, hk);
        if constexpr (K < 64) Dl = wrlane<K>(dk, Dl);
        else D2 = wrlane<K - 64>(dk, D2);
        if constexpr (S % 2 == 1) __builtin_amdgcn_sched_barrier(0);
        factor_steps<S + 1>(M, Dl, D2);
    }
}
template <int K>
__device__ __forceinline__ void factor(RegMat& M, float& Dl, float& D2, int) {
    factor_steps<0>(M, Dl, D2);
}

// ---------------------------------------------------------------- y <- L^-T y (y distributed: lane i holds y[i], y2 = y[64+i])
template <int K>
__device__ __forceinline__ void solve_LT(const RegMat& M, float& yl, float& y2, int lane) {
    if constexpr (K >= 1) {
        const float yk = K < 64 ? rdlane(yl, K) : rdlane(y2, K - 64);
        constexpr uint64_t lo = K < 64 ? (kAncLo[K] & ~(1ull << (K & 63))) : kAncLo[K];
        yl = lanes<lo>() ? yl - M.c[K] * yk : yl;
        if constexpr (K > 64) {
            constexpr uint64_t hi = kAncHi[K] & ~(1u << (K - 64));
            y2 = lanes<hi>() ? y2 - M.c2[K - 64] * yk : y2;
        }
        solve_LT<K - 1>(M, yl, y2, lane);
    }
}

// ---------------------------------------------------------------- y <- L^-1 y
template <int K>
__device__ __forceinline__ void solve_L(const RegMat& M, float& yl, float& y2, int lane) {
    if constexpr (K < NG) {
        float p = lane < K ? M.c[K] * yl : 0.0f;
        if constexpr (K > 64) p += lane < K - 64 ? M.c2[K - 64] * y2 : 0.0f;
        const float s = wave_sum(p);
        if constexpr (K < 64) {
            if (lane == K) yl -= s;
        } else {
            if (lane == K - 64) y2 -= s;
        }
        solve_L<K + 1>(M, yl, y2, lane);
    }
}

// ---------------------------------------------------------------- packed copy of L for broadcast reads
// Lp[kPackStart[K] + x] = L[K][kChain[K][x]] for x < depth(K) (rows padded to 4 floats): lane j
// writes the entries of its column j; pad slots are loaded but never used
template <int K>
__device__ __forceinline__ void store_packed(const RegMat& M, float* Lp, int lane, int lane_depth,
                                             int lane_depth2) {
    if constexpr (K >= 1) {
        constexpr uint64_t lo = K < 64 ? (kAncLo[K] & ~(1ull << (K & 63))) : kAncLo[K];
        if (lanes<lo>()) Lp[kPackStart[K] + lane_depth] = M.c[K];
        if constexpr (K > 64) {
            constexpr uint64_t hi = kAncHi[K] & ~(1u << (K - 64));
            if (lanes<hi>()) Lp[kPackStart[K] + lane_depth2] = M.c2[K - 64];
        }
        store_packed<K - 1>(M, Lp, lane, lane_depth, lane_depth2);
    }
}

// z -= a * b as an ordered instruction: the DAG linearisation would otherwise sink the whole
// unrolled sweep's FMAs below its LDS reads and spill the loaded rows
__device__ __forceinline__ void fnma(float& z, float a, float b) {
    asm volatile("v_fma_f32 %0, -%1, %2, %0" : "+v"(z) : "v"(a), "v"(b));
}

// ---------------------------------------------------------------- per-lane z <- L^-T z (each lane its own rhs)
// the packed row K (D entries) as registers: ceil(D/4) 16-byte LDS broadcasts
template <int D>
struct Row {
    float4 v[(D + 3) / 4 > 0 ? (D + 3) / 4 : 1];
};
template <int K>
__device__ __forceinline__ Row<kDofNanc[K] - 1> load_row(const float* Lp, int off) {
    Row<kDofNanc[K] - 1> r;
#pragma unroll
    for (int q = 0; q < (kDofNanc[K] - 1 + 3) / 4; ++q) r.v[q] = *reinterpret_cast<const float4*>(Lp + off + 4 * q);
    return r;
}
template <int K, int X, int D>
__device__ __forceinline__ void zbs_anc(const Row<D>& row, float (&z)[NG], float zk) {
    if constexpr (X < D) {
        const float4 v = row.v[X / 4];
        fnma(z[kChain[K][X]], v.x, zk);
        if constexpr (X + 1 < D) fnma(z[kChain[K][X + 1]], v.y, zk);
        if constexpr (X + 2 < D) fnma(z[kChain[K][X + 2]], v.z, zk);
        if constexpr (X + 3 < D) fnma(z[kChain[K][X + 3]], v.w, zk);
        zbs_anc<K, X + 4, D>(row, z, zk);
    }
}
// z <- L^-T z, one dof per step, software-pipelined: the next row is read (16-byte LDS
// broadcasts behind an opaque offset) while this one is applied. Only dofs of bodies
// in `lb` (the union of every row's ancestor bodies, wave-uniform) can be nonzero; the others are
// skipped without touching LDS.
template <int K>
__device__ __forceinline__ bool body_live(uint32_t lb) {
    if constexpr (K < 0) return false;
    else return (lb >> kDofBody[K]) & 1u;
}
template <int K>
struct RowOf {
    using T = Row<(K >= 0 ? kDofNanc[K < 0 ? 0 : K] : 1) - 1>;
};
template <int K>
__device__ __forceinline__ typename RowOf<K>::T load_row_if(const float* Lp, int off) {
    if constexpr (K >= 1) return load_row<K>(Lp, off + kPackStart[K]);
    else return typename RowOf<K>::T{};
}
// registers whose content does not matter (a row that is not loaded because its body is not live
// is never read): defined by an empty asm, so the compiler does not materialise zeros for them
__device__ __forceinline__ void undef_reg(float& x) { asm volatile("" : "=v"(x)); }
template <int D>
__device__ __forceinline__ void undef_row(Row<D>& r) {
#pragma unroll
    for (int q = 0; q < (D + 3) / 4 || q < 1; ++q) {
        undef_reg(r.v[q].x); undef_reg(r.v[q].y); undef_reg(r.v[q].z); undef_reg(r.v[q].w);
    }
}
template <int K>
__device__ __forceinline__ void zbs_pipe(const float* Lp, float (&z)[NG], uint32_t lb, const typename RowOf<K>::T& rk) {
    if constexpr (K >= 1) {
        typename RowOf<K - 1>::T nx;
        if constexpr (K - 1 >= 1) {
            if (body_live<K - 1>(lb)) {  // prefetch row K-1 while row K is applied
                int off = 0;
                asm volatile("" : "+v"(off));
                nx = load_row_if<K - 1>(Lp, off);
            } else {
                undef_row(nx);
            }
        }
        if (body_live<K>(lb)) zbs_anc<K, 0, kDofNanc[K] - 1>(rk, z, z[K]);
        __builtin_amdgcn_sched_barrier(0);
        zbs_pipe<K - 1>(Lp, z, lb, nx);
    }
}
template <int K>
__device__ __forceinline__ void zbs(const float* Lp, float (&z)[NG], uint32_t lb) {
    int off = 0;
    asm volatile("" : "+v"(off));
    const auto r0 = load_row_if<K>(Lp, off);
    zbs_pipe<K>(Lp, z, lb, r0);
}

// ---------------------------------------------------------------- y <- L^-1 y, row-distributed
// lane i holds row i of L as r1[x] = L[i][kChain[i][x]] (and r2 for dof 64+i); the position of an
// ancestor K in any chain through it is its depth, a compile-time constant, so each step is one
// v_readlane of y_K plus a masked FMA -- no cross-lane reduction.
constexpr int kRowRegs = 32;

// union over a depth level of the (disjoint) descendant lane sets
template <int D, int J = kLevelStart[D]>
constexpr uint64_t level_desc_lo() {
    if constexpr (J < kLevelStart[D + 1]) return kDescLo[kLevelDofs[J]] | level_desc_lo<D, J + 1>();
    else return 0ull;
}
template <int D, int J = kLevelStart[D]>
constexpr uint64_t level_desc_hi() {
    if constexpr (J < kLevelStart[D + 1]) return kDescHi[kLevelDofs[J]] | level_desc_hi<D, J + 1>();
    else return 0ull;
}
// per level: every descendant lane picks the y of its (unique) ancestor at this depth
template <int D, int J>
__device__ __forceinline__ void level_pick(float yl, float y2, float& t1, float& t2) {
    if constexpr (J < kLevelStart[D + 1]) {
        constexpr int K = kLevelDofs[J];
        if constexpr (kDescLo[K] != 0 || kDescHi[K] != 0) {
            const float yk = K < 64 ? rdlane(yl, K) : rdlane(y2, K - 64);
            if constexpr (kDescLo[K] != 0) t1 = lanes<kDescLo[K]>() ? yk : t1;
            if constexpr (kDescHi[K] != 0) t2 = lanes<(uint64_t)kDescHi[K]>() ? yk : t2;
        }
        level_pick<D, J + 1>(yl, y2, t1, t2);
    }
}
// y <- L^-1 y by depth levels, shallowest first: the dofs of one level have disjoint descendant
// sets, so a level is n readlanes + n selects + ONE fma with the row entry at that depth
template <int D>
__device__ __forceinline__ void solve_L_rows(const float (&r1)[kRowRegs], const float (&r2)[kRowRegs], float& yl,
                                             float& y2) {
    if constexpr (D < kNumLevels - 1) {
        constexpr uint64_t ulo = level_desc_lo<D>();
        constexpr uint64_t uhi = level_desc_hi<D>();
        if constexpr (ulo != 0 || uhi != 0) {
            float t1 = 0.f, t2 = 0.f;
            level_pick<D, kLevelStart[D]>(yl, y2, t1, t2);
            if constexpr (ulo != 0) yl = lanes<ulo>() ? yl - r1[D] * t1 : yl;
            if constexpr (uhi != 0) y2 = lanes<uhi>() ? y2 - r2[D] * t2 : y2;
        }
        solve_L_rows<D + 1>(r1, r2, yl, y2);
    }
}

// ---------------------------------------------------------------- y <- L^-T y, column-distributed
// by depth levels, deepest first. Lane j first gathers its whole column of L (g1[K] = L[K][j] =
// Lp[kPackStart[K] + depth(j)], 75 independent LDS reads issued back to back; entries of non-
// descendants are never selected), then each level is n readlanes of the final y_K plus n masked
// FMAs into an accumulator and one subtraction.
template <int K>
__device__ __forceinline__ void gather_cols(const float* Lp, int dj, int dj2, float (&g1)[NG], float (&g2)[NG - 64]) {
    if constexpr (K < NG) {
        if constexpr (K >= 1) g1[K] = Lp[kPackStart[K] + dj];
        if constexpr (K > 64) g2[K - 64] = Lp[kPackStart[K] + dj2];
        gather_cols<K + 1>(Lp, dj, dj2, g1, g2);
    }
}
template <int D, int J>
__device__ __forceinline__ void level_push(const float (&g1)[NG], const float (&g2)[NG - 64], float yl, float y2,
                                           float& t1, float& t2) {
    if constexpr (J < kLevelStart[D + 1]) {
        constexpr int K = kLevelDofs[J];
        if constexpr (K >= 1) {
            const float yk = K < 64 ? rdlane(yl, K) : rdlane(y2, K - 64);
            constexpr uint64_t lo = K < 64 ? (kAncLo[K] & ~(1ull << (K & 63))) : kAncLo[K];
            t1 = lanes<lo>() ? fmaf(g1[K], yk, t1) : t1;
            if constexpr (K > 64) {
                constexpr uint64_t hi = kAncHi[K] & ~(1u << (K - 64));
                t2 = lanes<hi>() ? fmaf(g2[K - 64], yk, t2) : t2;
            }
        }
        level_push<D, J + 1>(g1, g2, yl, y2, t1, t2);
    }
}
template <int D>
__device__ __forceinline__ void solve_LT_levels(const float (&g1)[NG], const float (&g2)[NG - 64], float& yl,
                                                float& y2) {
    if constexpr (D >= 1) {
        float t1 = 0.f, t2 = 0.f;
        level_push<D, kLevelStart[D]>(g1, g2, yl, y2, t1, t2);
        yl -= t1;
        y2 -= t2;
        solve_LT_levels<D - 1>(g1, g2, yl, y2);
    }
}
template <int D>
__device__ __forceinline__ void solve_LT_cols(const float* Lp, int dj, int dj2, float& yl, float& y2, int) {
    float g1[NG], g2[NG - 64];
    g1[0] = 0.f;
    g2[0] = 0.f;
    gather_cols<0>(Lp, dj, dj2, g1, g2);
    solve_LT_levels<D>(g1, g2, yl, y2);
}

// ---------------------------------------------------------------- LTDL with LDS row broadcasts
// As factor_steps, but row K of L leaves through LDS as soon as it is final (the packed store of
// the factor, lanes in chain(K) write their entry) and comes back as 16-byte broadcasts: the
// updates H[I][j] -= L[K][I] * H[K][j] then take both operands from VGPRs (one FMA, no v_readlane),
// halving the VALU work of the elimination. Leaves Lp complete (no separate store_packed).
template <int K, int X, int D>
__device__ __forceinline__ void fac_anc_row(RegMat& M, const Row<D>& row, float t, float t2) {
    if constexpr (X < D) {
        constexpr int I = kChain[K][X];
        const float4 v = row.v[X / 4];
        const float l = (X % 4 == 0) ? v.x : ((X % 4 == 1) ? v.y : ((X % 4 == 2) ? v.z : v.w));
        fnma(M.c[I], l, t);  // ordered: keeps the row's registers short-lived
        if constexpr (I >= 64) fnma(M.c2[I - 64], l, t2);
        fac_anc_row<K, X + 1, D>(M, row, t, t2);
    }
}
template <int S>
__device__ __forceinline__ void factor_lds_steps(RegMat& M, float& Dl, float& D2, float* Lp, int dj, int dj2,
                                                 float& yl, float& y2) {
    if constexpr (S < NG) {
        constexpr int K = kElimOrder[S];
        constexpr int D = kDofNanc[K] - 1;
        const float dk = get<K, K>(M);
        const float inv = uniform(__builtin_amdgcn_rcpf(dk));
        const float t = M.c[K];                        // H[K][j], unscaled
        const float t2 = K >= 64 ? M.c2[K >= 64 ? K - 64 : 0] : 0.f;
        M.c[K] = t * inv;                              // L[K][j] on lanes j < K
        if constexpr (K >= 64) M.c2[K - 64] = t2 * inv;
        if constexpr (D > 0) {
            constexpr uint64_t lo = K < 64 ? (kAncLo[K] & ~(1ull << (K & 63))) : kAncLo[K];
            // forward substitution of the right-hand side fused in (y = L^-T rhs, the same
            // deepest-first order): y[K] is final once K's descendants are eliminated
            const float yk = K < 64 ? rdlane(yl, K) : rdlane(y2, K >= 64 ? K - 64 : 0);
            if (lanes<lo>()) {
                Lp[kPackStart[K] + dj] = M.c[K];
                yl = yl - M.c[K] * yk;
            }
            if constexpr (K > 64) {
                constexpr uint64_t hi = kAncHi[K] & ~(1u << (K - 64));
                if (lanes<hi>()) {
                    Lp[kPackStart[K] + dj2] = M.c2[K - 64];
                    y2 = y2 - M.c2[K - 64] * yk;
                }
            }
            const auto row = load_row<K>(Lp, kPackStart[K]);  // in-order LDS: sees the writes above
            fac_anc_row<K, 0, D>(M, row, t, t2);
        }
        if constexpr (K < 64) Dl = wrlane<K>(dk, Dl);
        else D2 = wrlane<K - 64>(dk, D2);
        __builtin_amdgcn_sched_barrier(0);
        factor_lds_steps<S + 1>(M, Dl, D2, Lp, dj, dj2, yl, y2);
    }
}

// ---------------------------------------------------------------- grouped elimination
// Consecutive steps of kElimOrder whose dofs are mutually independent (neither is an ancestor of
// the other: different branches) touch disjoint pivots and rows, so a group of them runs as one
// step: all pivots and reciprocals, then all packed-row stores and right-hand-side updates, then
// all row broadcasts (one LDS round trip), then the ancestor updates in the original order. Every
// register sees its updates in the same order as in the one-at-a-time elimination, so the factor
// is bit-identical to factor_lds_steps; the dependent latency chain is paid once per group.
constexpr bool dof_is_anc(int a, int b) {  // b in chain(a), a itself included
    return b < 64 ? ((kAncLo[a] >> b) & 1ull) != 0 : ((kAncHi[a] >> (b - 64)) & 1u) != 0;
}
template <int GMAX>
struct ElimGroups {
    int start[NG + 1];
    int count;
    constexpr ElimGroups() : start(), count(0) {
        int i = 0;
        while (i < NG) {
            start[count++] = i;
            int j = i + 1;
            while (j < NG && j - i < GMAX) {
                bool ok = true;
                for (int x = i; x < j; ++x)
                    if (dof_is_anc(kElimOrder[j], kElimOrder[x]) || dof_is_anc(kElimOrder[x], kElimOrder[j])) ok = false;
                if (!ok) break;
                ++j;
            }
            i = j;
        }
        start[count] = NG;
    }
};
constexpr int kElimGroupMax = 2;
constexpr ElimGroups<kElimGroupMax> kElimGroups{};

template <int K>
struct PivotStep {
    float dk, t, t2;
    Row<kDofNanc[K] - 1> row;
};
// A: pivot, reciprocal, row K of L on lanes j < K
template <int K>
__device__ __forceinline__ void grp_pivot(RegMat& M, PivotStep<K>& st) {
    st.dk = get<K, K>(M);
    const float inv = uniform(__builtin_amdgcn_rcpf(st.dk));
    st.t = M.c[K];
    st.t2 = K >= 64 ? M.c2[K >= 64 ? K - 64 : 0] : 0.f;
    M.c[K] = st.t * inv;
    if constexpr (K >= 64) M.c2[K - 64] = st.t2 * inv;
}
// B: packed-row store and the fused forward substitution of the right-hand side
template <int K>
__device__ __forceinline__ void grp_store(const RegMat& M, float* Lp, int dj, int dj2, float& yl, float& y2) {
    if constexpr (kDofNanc[K] - 1 > 0) {
        constexpr uint64_t lo = K < 64 ? (kAncLo[K] & ~(1ull << (K & 63))) : kAncLo[K];
        const float yk = K < 64 ? rdlane(yl, K) : rdlane(y2, K >= 64 ? K - 64 : 0);
        if (lanes<lo>()) {
            Lp[kPackStart[K] + dj] = M.c[K];
            yl = yl - M.c[K] * yk;
        }
        if constexpr (K > 64) {
            constexpr uint64_t hi = kAncHi[K] & ~(1u << (K - 64));
            if (lanes<hi>()) {
                Lp[kPackStart[K] + dj2] = M.c2[K - 64];
                y2 = y2 - M.c2[K - 64] * yk;
            }
        }
    }
}
// C + D: row broadcast (in-order LDS: sees the stores of B) and the ancestor updates
template <int K>
__device__ __forceinline__ void grp_load(const float* Lp, PivotStep<K>& st) {
    if constexpr (kDofNanc[K] - 1 > 0) st.row = load_row<K>(Lp, kPackStart[K]);
}
template <int K>
__device__ __forceinline__ void grp_update(RegMat& M, float& Dl, float& D2, const PivotStep<K>& st) {
    if constexpr (kDofNanc[K] - 1 > 0) fac_anc_row<K, 0, kDofNanc[K] - 1>(M, st.row, st.t, st.t2);
    if constexpr (K < 64) Dl = wrlane<K>(st.dk, Dl);
    else D2 = wrlane<K - 64>(st.dk, D2);
}
template <int GI>
__device__ __forceinline__ void factor_lds_groups(RegMat& M, float& Dl, float& D2, float* Lp, int dj, int dj2,
                                                  float& yl, float& y2) {
    if constexpr (GI < kElimGroups.count) {
        constexpr int S0 = kElimGroups.start[GI], n = kElimGroups.start[GI + 1] - S0;
        static_assert(n >= 1 && n <= 3, "group size");
        constexpr int K0 = kElimOrder[S0];
        constexpr int K1 = kElimOrder[n > 1 ? S0 + 1 : S0];
        constexpr int K2 = kElimOrder[n > 2 ? S0 + 2 : S0];
        PivotStep<K0> a;
        PivotStep<K1> b;
        PivotStep<K2> c;
        grp_pivot<K0>(M, a);
        if constexpr (n > 1) grp_pivot<K1>(M, b);
        if constexpr (n > 2) grp_pivot<K2>(M, c);
        grp_store<K0>(M, Lp, dj, dj2, yl, y2);
        if constexpr (n > 1) grp_store<K1>(M, Lp, dj, dj2, yl, y2);
        if constexpr (n > 2) grp_store<K2>(M, Lp, dj, dj2, yl, y2);
        grp_load<K0>(Lp, a);
        if constexpr (n > 1) grp_load<K1>(Lp, b);
        if constexpr (n > 2) grp_load<K2>(Lp, c);
        grp_update<K0>(M, Dl, D2, a);
        if constexpr (n > 1) grp_update<K1>(M, Dl, D2, b);
        if constexpr (n > 2) grp_update<K2>(M, Dl, D2, c);
        __builtin_amdgcn_sched_barrier(0);
        factor_lds_groups<GI + 1>(M, Dl, D2, Lp, dj, dj2, yl, y2);
    }
}
}  // namespace regla
