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

typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));

// c[i] = cp[i >> 1][i & 1], c2[i] = cp2[i >> 1][i & 1]: dofs (2k, 2k+1) share an aligned VGPR pair,
// so two updates with a common multiplier are one v_pk_fma_f32
struct RegMat {
    f2v cp[(NG + 1) / 2];
    f2v cp2[(NH + 1) / 2];
};
template <int I>
__device__ __forceinline__ float mc(const RegMat& M) { return M.cp[I >> 1][I & 1]; }
template <int I>
__device__ __forceinline__ void mc_set(RegMat& M, float v) { M.cp[I >> 1][I & 1] = v; }
template <int I>
__device__ __forceinline__ float mc2(const RegMat& M) { return M.cp2[I >> 1][I & 1]; }
template <int I>
__device__ __forceinline__ void mc2_set(RegMat& M, float v) { M.cp2[I >> 1][I & 1] = v; }

__device__ __forceinline__ float rdlane(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// lanes L .. L+3 of v into four SGPRs in one block: the allocator otherwise routes every broadcast of
// a dot product through one SGPR, each behind its own hazard nop, and the products serialise
template <int L>
__device__ __forceinline__ void rdlane4(float v, float (&s)[4]) {
    asm volatile(
        "s_nop 0\n"
        "v_readlane_b32 %0, %4, %5\n"
        "v_readlane_b32 %1, %4, %6\n"
        "v_readlane_b32 %2, %4, %7\n"
        "v_readlane_b32 %3, %4, %8\n"
        "s_nop 1"
        : "=s"(s[0]), "=s"(s[1]), "=s"(s[2]), "=s"(s[3])
        : "v"(v), "i"(L), "i"(L + 1), "i"(L + 2), "i"(L + 3));
}

// f(integral_constant<I>) for I = I0, I0 + STEP, ... < N (compile-time lane indices for rdlane4)
template <int I0, int N, int STEP, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (I0 < N) {
        f(std::integral_constant<int, I0>{});
        static_for<I0 + STEP, N, STEP>(f);
    }
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
    if constexpr (COL < 64) return rdlane(mc<ROW>(M), COL);
    else return rdlane(mc2<ROW - 64>(M), COL - 64);
}

// lanes whose bit is set in the compile-time mask C (v_cndmask on an SGPR-pair constant; no
// per-lane compare or branch)
template <uint64_t C>
__device__ __forceinline__ bool lanes() {
    // the constant is materialised here by two s_mov_b32 (volatile: never hoisted out of the
    // substep loop, where dozens of distinct masks would otherwise be kept live and spilled)
#ifndef HE_LANES_B64
#define HE_LANES_B64 1
#endif
#ifndef HE_LANES_BFM
#define HE_LANES_BFM 1
#endif
    constexpr int kOff = C == 0 ? 0 : __builtin_ctzll(C);
    constexpr int kLen = C == 0 ? 0 : 64 - __builtin_clzll(C) - kOff;
    constexpr bool kRun = C != 0 && kLen < 64 && C == (((1ull << kLen) - 1ull) << kOff);
    if constexpr (HE_LANES_BFM && kRun) {
        // a run of lanes (descendant sets are runs in the DFS dof order): one s_bfm_b64 of two
        // inline constants, ((1 << len) - 1) << off
        uint64_t m;
        asm volatile("s_bfm_b64 %0, %1, %2" : "=s"(m) : "i"(kLen), "i"(kOff));
        return __builtin_amdgcn_inverse_ballot_w64(m);
    } else if constexpr (HE_LANES_B64 && C < 0x80000000ull) {
        // lanes < 31 only: one s_mov_b64 of a non-negative 32-bit constant (a 64-bit SALU move
        // zero-extends its 32-bit literal, so a mask with lanes >= 32 set needs the pair)
        uint64_t m;
        asm volatile("s_mov_b64 %0, %1" : "=s"(m) : "i"((int32_t)(uint32_t)C));
        return __builtin_amdgcn_inverse_ballot_w64(m);
    } else {
        uint32_t lo, hi;
        asm volatile("s_mov_b32 %0, %1" : "=s"(lo) : "i"((uint32_t)C));
        asm volatile("s_mov_b32 %0, %1" : "=s"(hi) : "i"((uint32_t)(C >> 32)));
        return __builtin_amdgcn_inverse_ballot_w64(((uint64_t)hi << 32) | lo);
    }
}

// z -= a * b as an ordered instruction: the DAG linearisation would otherwise sink the whole
// unrolled sweep's FMAs below its LDS reads and spill the loaded rows
__device__ __forceinline__ void fnma(float& z, float a, float b) {
    asm volatile("v_fma_f32 %0, -%1, %2, %0" : "+v"(z) : "v"(a), "v"(b));
}

// z, z' -= a * b, a' * b as one v_pk_fma_f32, b taken from half HALF of its register pair
template <int HALF>
__device__ __forceinline__ void pk_fnma(f2v& z, f2v a, f2v b) {
    if constexpr (HALF == 0)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1] neg_lo:[1,0,0] neg_hi:[1,0,0]"
                     : "+v"(z) : "v"(a), "v"(b));
    else
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[1,1,1] neg_lo:[1,0,0] neg_hi:[1,0,0]"
                     : "+v"(z) : "v"(a), "v"(b));
}

// ---------------------------------------------------------------- LTDL factorisation and solves
// ---------------------------------------------------------------- per-lane z <- L^-T z (each lane its own rhs)
// the packed row K (D entries) as registers: ceil(D/4) 16-byte LDS broadcasts
template <int D>
struct Row {
    f4v v[(D + 3) / 4 > 0 ? (D + 3) / 4 : 1];
};
template <int K>
__device__ __forceinline__ Row<kDofNanc[K] - 1> load_row(const float* Lp, int off) {
    Row<kDofNanc[K] - 1> r;
#pragma unroll
    for (int q = 0; q < (kDofNanc[K] - 1 + 3) / 4; ++q) r.v[q] = *reinterpret_cast<const f4v*>(Lp + off + 4 * q);
    return r;
}
// a contact row's dof vector, dofs (2k, 2k+1) in one aligned register pair
struct ZVec {
    f2v p[(NG + 1) / 2];
};
#define ZV(z, i) (z).p[(i) >> 1][(i) & 1]

template <int K, int X, int D>
__device__ __forceinline__ void zbs_anc(const Row<D>& row, ZVec& z) {
    if constexpr (X < D) {
        constexpr int I = kChain[K][X];
        constexpr bool PAIR = X % 2 == 0 && X + 1 < D && I % 2 == 0 && kChain[K][X + 1 < kMaxChain ? X + 1 : 0] == I + 1;
        const f4v v = row.v[X / 4];
        if constexpr (PAIR) {  // z[I], z[I+1] -= L[K][I], L[K][I+1] * z[K]: one v_pk_fma_f32
            const f2v l = X % 4 == 0 ? __builtin_shufflevector(v, v, 0, 1) : __builtin_shufflevector(v, v, 2, 3);
            pk_fnma<K & 1>(z.p[I >> 1], l, z.p[K >> 1]);
            zbs_anc<K, X + 2, D>(row, z);
        } else {
            const float l = (X % 4 == 0) ? v.x : ((X % 4 == 1) ? v.y : ((X % 4 == 2) ? v.z : v.w));
            float t = ZV(z, I);
            fnma(t, l, ZV(z, K));
            ZV(z, I) = t;
            zbs_anc<K, X + 1, D>(row, z);
        }
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
        asm volatile("" : "=v"(r.v[q]));
    }
}
// body-level variant: one liveness branch per body (its 3 rows, or the root's 5, applied in a
// row-prefetch chain inside it) instead of two per dof
template <int K>
constexpr int dof_first_of_body() { return K < 6 ? 0 : 6 + 3 * ((K - 6) / 3); }
template <int K>
__device__ __forceinline__ typename RowOf<K>::T row_if_live(const float* Lp, uint32_t lb) {
    typename RowOf<K>::T r;
    if constexpr (K >= 1) {
        if (body_live<K>(lb)) {
            r = load_row_if<K>(Lp, 0);  // the callers' sched_barriers keep it where it is issued
        } else {
            undef_row(r);
        }
    } else {
        undef_row(r);
    }
    return r;
}
// rows K .. K0 of one live body: row K is in registers, row K-1 (same body) is requested first
template <int K, int K0>
__device__ __forceinline__ void zbs_in_body(const float* Lp, ZVec& z, const typename RowOf<K>::T& rk) {
    if constexpr (K > K0 && K >= 1) {
        // the next row's broadcast, issued before this row's updates; the sched_barrier after them
        // keeps it here (no opaque offset: its address arithmetic cost 2 VALU per row)
        const typename RowOf<K - 1>::T nx = load_row_if<K - 1>(Lp, 0);
        zbs_anc<K, 0, kDofNanc[K] - 1>(rk, z);
        __builtin_amdgcn_sched_barrier(0);
        zbs_in_body<K - 1, K0>(Lp, z, nx);
    } else if constexpr (K >= 1) {
        zbs_anc<K, 0, kDofNanc[K] - 1>(rk, z);
        __builtin_amdgcn_sched_barrier(0);
    }
}
template <int K>  // K: the last dof of a body (74, 71, ..., 8, then 5 for the root)
__device__ __forceinline__ void zbs_bodies(const float* Lp, ZVec& z, uint32_t lb, const typename RowOf<K>::T& rk) {
    if constexpr (K >= 1) {
        constexpr int K0 = dof_first_of_body<K>();
        if (body_live<K>(lb)) zbs_in_body<K, K0>(Lp, z, rk);
        // the next body's last row (requested after this body's updates were issued)
        const typename RowOf<K0 - 1>::T nx = row_if_live<K0 - 1>(Lp, lb);
        __builtin_amdgcn_sched_barrier(0);
        zbs_bodies<K0 - 1>(Lp, z, lb, nx);
    }
}

template <int K>
__device__ __forceinline__ void zbs(const float* Lp, ZVec& z, uint32_t lb) {
    zbs_bodies<K>(Lp, z, lb, row_if_live<K>(Lp, lb));
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
// per level: every descendant lane picks the y of its (unique) ancestor at this depth. The first
// dof of the level with descendants in a register set is written to every lane of it (a plain
// broadcast, no select): the caller's update is restricted to the level's descendant lanes, so what
// the others hold does not matter, and t1 / t2 need no zero fill
template <int D, int J, bool F1 = true, bool F2 = true>
__device__ __forceinline__ void level_pick(float yl, float y2, float& t1, float& t2) {
    if constexpr (J < kLevelStart[D + 1]) {
        constexpr int K = kLevelDofs[J];
        if constexpr (kDescLo[K] != 0 || kDescHi[K] != 0) {
            const float yk = K < 64 ? rdlane(yl, K) : rdlane(y2, K - 64);
            if constexpr (kDescLo[K] != 0) t1 = F1 ? yk : (lanes<kDescLo[K]>() ? yk : t1);
            if constexpr (kDescHi[K] != 0) t2 = F2 ? yk : (lanes<(uint64_t)kDescHi[K]>() ? yk : t2);
        }
        level_pick<D, J + 1, F1 && kDescLo[K] == 0, F2 && kDescHi[K] == 0>(yl, y2, t1, t2);
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
            float t1, t2;  // written by level_pick on every lane of a set the level touches
            undef_reg(t1);
            undef_reg(t2);
            level_pick<D, kLevelStart[D]>(yl, y2, t1, t2);
            if constexpr (ulo != 0) yl = lanes<ulo>() ? yl - r1[D] * t1 : yl;
            if constexpr (uhi != 0) y2 = lanes<uhi>() ? y2 - r2[D] * t2 : y2;
        }
        solve_L_rows<D + 1>(r1, r2, yl, y2);
    }
}

// the same sweep with the packed rows streamed from LDS four levels at a time, one 16-byte block a
// level-group ahead (16 registers instead of solve_L_rows' 64 preloaded): for phases where the rows
// compete with long-lived state for registers (the TGS iterations' velocity updates). p1 / p2: the
// lane's rows of dof lane and dof 64 + lane (16-byte aligned, as load_rows); only entries below the
// dof's depth are used, as in solve_L_rows.
template <int D>
__device__ __forceinline__ void solve_L_stream(const f4v* p1, const f4v* p2, f4v c1, f4v c2, f4v n1, f4v n2, float& yl,
                                               float& y2) {
    if constexpr (D < kNumLevels - 1) {
        if constexpr (D > 0 && D % 4 == 0) {
            c1 = n1;
            c2 = n2;
            if constexpr (D / 4 + 1 < kRowRegs / 4) {
                int off = 0;
                asm volatile("" : "+v"(off));  // the next block's loads stay here, a group ahead
                n1 = *reinterpret_cast<const f4v*>(reinterpret_cast<const char*>(p1 + D / 4 + 1) + off);
                n2 = *reinterpret_cast<const f4v*>(reinterpret_cast<const char*>(p2 + D / 4 + 1) + off);
            }
        }
        constexpr uint64_t ulo = level_desc_lo<D>();
        constexpr uint64_t uhi = level_desc_hi<D>();
        if constexpr (ulo != 0 || uhi != 0) {
            float t1, t2;  // written by level_pick on every lane of a set the level touches
            undef_reg(t1);
            undef_reg(t2);
            level_pick<D, kLevelStart[D]>(yl, y2, t1, t2);
            if constexpr (ulo != 0) yl = lanes<ulo>() ? yl - c1[D % 4] * t1 : yl;
            if constexpr (uhi != 0) y2 = lanes<uhi>() ? y2 - c2[D % 4] * t2 : y2;
        }
        solve_L_stream<D + 1>(p1, p2, c1, c2, n1, n2, yl, y2);
    }
}
__device__ __forceinline__ void solve_L_streamed(const float* row1, const float* row2, float& yl, float& y2) {
    const f4v* p1 = reinterpret_cast<const f4v*>(row1);
    const f4v* p2 = reinterpret_cast<const f4v*>(row2);
    solve_L_stream<0>(p1, p2, p1[0], p2[0], p1[1], p2[1], yl, y2);
}

// ---------------------------------------------------------------- y <- L^-T y, one vector
// Lane j holds y_j (and y_{64+j} in y2). The elimination's forward substitution replayed from the
// stored factor: pivots in kElimOrder (deepest first, so every descendant of K is final before K
// is read), each ancestor j of K taking y_j -= L[K][j] y_K with L[K][j] = Lp[kPackStart[K] + depth(j)].
// Used by the midpoint bias's correction, once per substep (not on the factor's latency chain).
// The pivots run in groups of mutually independent ones (no pivot of a group is an ancestor of
// another, so every y_K of a group is final when the group starts; ElimGroups below): the group's
// broadcasts are read first, then its updates, so the dependent chain is paid once per group
// instead of once per pivot.
template <int GMAX>
struct ElimGroups;
template <int S0, int Q, int N>
__device__ __forceinline__ void lt_group_read(float (&yk)[N], float yl, float y2) {
    if constexpr (Q < N) {
        constexpr int K = kElimOrder[S0 + Q];
        yk[Q] = K < 64 ? rdlane(yl, K) : rdlane(y2, K >= 64 ? K - 64 : 0);
        lt_group_read<S0, Q + 1, N>(yk, yl, y2);
    }
}

// ---------------------------------------------------------------- grouped elimination
// Consecutive steps of kElimOrder whose dofs are mutually independent (neither is an ancestor of
// the other: different branches) touch disjoint pivots and rows, so a group of them runs as one
// step: all pivots and reciprocals, then all packed-row stores and right-hand-side updates, then
// all row broadcasts (one LDS round trip), then the ancestor updates in the original order. Every
// register sees its updates in the same order as in the one-at-a-time elimination, so the factor
// is bit-identical to the one-at-a-time elimination; the dependent latency chain is paid once per group.
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

// The packed-row loads run one group ahead: group G+1's L entries are read (every lane, its own
// ancestor offset, clamped into the factor) while group G's pivots are broadcast and applied, so a
// group (of at most 4 pivots) pays its readlanes and FMAs but not an LDS round trip. The update
// stays exec-masked to the pivot's ancestor lanes.
constexpr ElimGroups<4> kLTPipeGroups{};
template <int G>
struct LTGroup {
    static constexpr int S0 = G < kLTPipeGroups.count ? kLTPipeGroups.start[G] : 0;
    static constexpr int N = G < kLTPipeGroups.count ? kLTPipeGroups.start[G + 1] - S0 : 1;
};
// p1 = Lp + dj, p2 = Lp + dj2 (the lane's depth offsets, added once per group): each entry is one LDS
// read at an immediate offset, no per-pivot address arithmetic. A lane that is not an ancestor of
// K reads past row K (other rows of the factor, or the words after it); lt_group_apply's select
// never lets that value in.
template <int S0, int Q, int N>
__device__ __forceinline__ void lt_group_load(const float* p1, const float* p2, float (&l1)[N], float (&l2)[N]) {
    if constexpr (Q < N) {
        constexpr int K = kElimOrder[S0 + Q];
        if constexpr (kDofNanc[K] - 1 > 0) {
            l1[Q] = p1[kPackStart[K]];
            if constexpr (K > 64) l2[Q] = p2[kPackStart[K]];
        }
        lt_group_load<S0, Q + 1, N>(p1, p2, l1, l2);
    }
}
template <int S0, int Q, int N>
__device__ __forceinline__ void lt_group_apply(const float (&l1)[N], const float (&l2)[N], const float (&yk)[N],
                                               float& yl, float& y2) {
    if constexpr (Q < N) {
        constexpr int K = kElimOrder[S0 + Q];
        if constexpr (kDofNanc[K] - 1 > 0) {
            constexpr uint64_t lo = K < 64 ? (kAncLo[K] & ~(1ull << (K & 63))) : kAncLo[K];
            if (lanes<lo>()) yl = yl - l1[Q] * yk[Q];
            if constexpr (K > 64) {
                constexpr uint64_t hi = kAncHi[K] & ~(1u << (K - 64));
                if (lanes<hi>()) y2 = y2 - l2[Q] * yk[Q];
            }
        }
        lt_group_apply<S0, Q + 1, N>(l1, l2, yk, yl, y2);
    }
}
template <int G>
__device__ __forceinline__ void solve_LT_vec_pipe(const float* Lp, int dj, int dj2, float& yl, float& y2,
                                                  const float (&l1)[LTGroup<G>::N], const float (&l2)[LTGroup<G>::N]) {
    if constexpr (G < kLTPipeGroups.count) {
        using C = LTGroup<G>;
        using Nx = LTGroup<G + 1>;
        float n1[Nx::N], n2[Nx::N];
        if constexpr (G + 1 < kLTPipeGroups.count) {
            // the loads stay here, one group ahead: the group's sched_barrier below keeps them in
            // this region (no opaque offset: its per-group address arithmetic cost 4 VALU)
            lt_group_load<Nx::S0, 0, Nx::N>(Lp + dj, Lp + dj2, n1, n2);
        }
        float yk[C::N];
        lt_group_read<C::S0, 0, C::N>(yk, yl, y2);
        lt_group_apply<C::S0, 0, C::N>(l1, l2, yk, yl, y2);
        __builtin_amdgcn_sched_barrier(0);
        solve_LT_vec_pipe<G + 1>(Lp, dj, dj2, yl, y2, n1, n2);
    }
}
__device__ __forceinline__ void solve_LT_vec_pipelined(const float* Lp, int dj, int dj2, float& yl, float& y2) {
    float l1[LTGroup<0>::N], l2[LTGroup<0>::N];
    lt_group_load<LTGroup<0>::S0, 0, LTGroup<0>::N>(Lp + dj, Lp + dj2, l1, l2);
    solve_LT_vec_pipe<0>(Lp, dj, dj2, yl, y2, l1, l2);
}

template <int K>
struct PivotStep {
    float dk, l, l2;  // pivot, row K of L on this lane (scaled) and its second-set entry
    Row<kDofNanc[K] - 1> row;
};
// A: pivot and reciprocal; the scaled entry L[K][j] goes to a fresh register, M keeps the unscaled
// H[K][j] as the broadcast operand of the updates until grp_finish
template <int K>
__device__ __forceinline__ void grp_pivot(const RegMat& M, PivotStep<K>& st) {
    st.dk = get<K, K>(M);
    const float inv = __builtin_amdgcn_rcpf(st.dk);
    st.l = mc<K>(M) * inv;
    if constexpr (K >= 64) st.l2 = mc2<K >= 64 ? K - 64 : 0>(M) * inv;
}
// B: packed-row store and the fused forward substitution of the right-hand side
template <int K>
__device__ __forceinline__ void grp_store(const PivotStep<K>& st, float* Lp, int dj, int dj2, float& yl, float& y2) {
    if constexpr (kDofNanc[K] - 1 > 0) {
        constexpr uint64_t lo = K < 64 ? (kAncLo[K] & ~(1ull << (K & 63))) : kAncLo[K];
        const float yk = K < 64 ? rdlane(yl, K) : rdlane(y2, K >= 64 ? K - 64 : 0);
        if (lanes<lo>()) {
            Lp[kPackStart[K] + dj] = st.l;
            yl = yl - st.l * yk;
        }
        if constexpr (K > 64) {
            constexpr uint64_t hi = kAncHi[K] & ~(1u << (K - 64));
            if (lanes<hi>()) {
                Lp[kPackStart[K] + dj2] = st.l2;
                y2 = y2 - st.l2 * yk;
            }
        }
    }
}
template <int K, int I>
__device__ __forceinline__ float lrow(const PivotStep<K>& st) {  // L[K][I], wave-uniform
    if constexpr (I < 64) return rdlane(st.l, I);
    else return rdlane(st.l2, I >= 64 ? I - 64 : 0);
}
// ---------------------------------------------------------------- software-pipelined groups
// The next group's pivots only wait for the updates of their own rows. Those rows (I in chain(K)
// and a pivot of group GI+1) take L[K][I] straight from lane I (one v_readlane) as soon as row K
// is scaled; group GI+1 is then pivoted, stored and its LDS broadcast issued before group GI's
// remaining updates wait for theirs. Every register still sees its updates in elimination order,
// so the factor is bit-identical.
template <int G>
constexpr bool in_group(int I) {
    if (G >= kElimGroups.count) return false;
    for (int x = kElimGroups.start[G]; x < kElimGroups.start[G + 1]; ++x)
        if (kElimOrder[x] == I) return true;
    return false;
}
template <int K, int X, int D, int GN>
__device__ __forceinline__ void fac_anc_fast(RegMat& M, const PivotStep<K>& st) {
    if constexpr (X < D) {
        constexpr int I = kChain[K][X];
        if constexpr (in_group<GN>(I)) {
            const float l = lrow<K, I>(st);
            float c = mc<I>(M);
            fnma(c, l, mc<K>(M));
            mc_set<I>(M, c);
            if constexpr (I >= 64) {
                float c2 = mc2<I - 64>(M);
                fnma(c2, l, mc2<K >= 64 ? K - 64 : 0>(M));
                mc2_set<I - 64>(M, c2);
            }
        }
        fac_anc_fast<K, X + 1, D, GN>(M, st);
    }
}
template <int K, int X, int D, int GN>
__device__ __forceinline__ void fac_anc_slow(RegMat& M, const Row<D>& row) {
    if constexpr (X < D) {
        constexpr int I = kChain[K][X];
        constexpr bool FAST = in_group<GN>(I);
        constexpr bool PAIR = !FAST && X % 2 == 0 && X + 1 < D && I % 2 == 0 && I + 1 < 64 &&
                              kChain[K][X + 1 < kMaxChain ? X + 1 : 0] == I + 1 && !in_group<GN>(I + 1);
        const f4v v = row.v[X / 4];
        if constexpr (FAST) {
            fac_anc_slow<K, X + 1, D, GN>(M, row);
        } else if constexpr (PAIR) {
            const f2v l = X % 4 == 0 ? __builtin_shufflevector(v, v, 0, 1) : __builtin_shufflevector(v, v, 2, 3);
            pk_fnma<K & 1>(M.cp[I >> 1], l, M.cp[K >> 1]);
            fac_anc_slow<K, X + 2, D, GN>(M, row);
        } else {
            const float l = (X % 4 == 0) ? v.x : ((X % 4 == 1) ? v.y : ((X % 4 == 2) ? v.z : v.w));
            float c = mc<I>(M);
            fnma(c, l, mc<K>(M));
            mc_set<I>(M, c);
            if constexpr (I >= 64) {
                float c2 = mc2<I - 64>(M);
                fnma(c2, l, mc2<K >= 64 ? K - 64 : 0>(M));
                mc2_set<I - 64>(M, c2);
            }
            fac_anc_slow<K, X + 1, D, GN>(M, row);
        }
    }
}
template <int GI>
struct GSteps {
    static constexpr int S0 = kElimGroups.start[GI < kElimGroups.count ? GI : 0];
    static constexpr int n = GI < kElimGroups.count ? kElimGroups.start[GI + 1] - S0 : 1;
    static constexpr int K0 = kElimOrder[S0];
    static constexpr int K1 = kElimOrder[n > 1 ? S0 + 1 : S0];
    static constexpr int K2 = kElimOrder[n > 2 ? S0 + 2 : S0];
    PivotStep<K0> a;
    PivotStep<K1> b;
    PivotStep<K2> c;
};
template <int K>
__device__ __forceinline__ void grp_load_always(const float* Lp, PivotStep<K>& st) {
    if constexpr (kDofNanc[K] - 1 > 0) st.row = load_row<K>(Lp, kPackStart[K]);
}
template <int GI>
__device__ __forceinline__ void group_front(RegMat& M, GSteps<GI>& g, float* Lp, int dj, int dj2, float& yl, float& y2) {
    using G = GSteps<GI>;
    grp_pivot<G::K0>(M, g.a);
    if constexpr (G::n > 1) grp_pivot<G::K1>(M, g.b);
    if constexpr (G::n > 2) grp_pivot<G::K2>(M, g.c);
    grp_store<G::K0>(g.a, Lp, dj, dj2, yl, y2);
    if constexpr (G::n > 1) grp_store<G::K1>(g.b, Lp, dj, dj2, yl, y2);
    if constexpr (G::n > 2) grp_store<G::K2>(g.c, Lp, dj, dj2, yl, y2);
    grp_load_always<G::K0>(Lp, g.a);
    if constexpr (G::n > 1) grp_load_always<G::K1>(Lp, g.b);
    if constexpr (G::n > 2) grp_load_always<G::K2>(Lp, g.c);
}
template <int K, int GN>
__device__ __forceinline__ void grp_finish(RegMat& M, float& Dl, float& D2, const PivotStep<K>& st) {
    if constexpr (kDofNanc[K] - 1 > 0) fac_anc_slow<K, 0, kDofNanc[K] - 1, GN>(M, st.row);
    mc_set<K>(M, st.l);  // row K -> L[K][.] on lanes j < K
    if constexpr (K >= 64) mc2_set<K - 64>(M, st.l2);
    if constexpr (K < 64) Dl = wrlane<K>(st.dk, Dl);
    else D2 = wrlane<K - 64>(st.dk, D2);
}
template <int GI>
__device__ __forceinline__ void factor_pipe(RegMat& M, float& Dl, float& D2, float* Lp, int dj, int dj2, float& yl,
                                            float& y2, GSteps<GI>& g) {
    if constexpr (GI < kElimGroups.count) {
        using G = GSteps<GI>;
        constexpr int GN = GI + 1;
        if constexpr (kDofNanc[G::K0] - 1 > 0) fac_anc_fast<G::K0, 0, kDofNanc[G::K0] - 1, GN>(M, g.a);
        if constexpr (G::n > 1 && kDofNanc[G::K1] - 1 > 0) fac_anc_fast<G::K1, 0, kDofNanc[G::K1] - 1, GN>(M, g.b);
        if constexpr (G::n > 2 && kDofNanc[G::K2] - 1 > 0) fac_anc_fast<G::K2, 0, kDofNanc[G::K2] - 1, GN>(M, g.c);
        GSteps<GN> gn;
        if constexpr (GN < kElimGroups.count) group_front<GN>(M, gn, Lp, dj, dj2, yl, y2);
        grp_finish<G::K0, GN>(M, Dl, D2, g.a);
        if constexpr (G::n > 1) grp_finish<G::K1, GN>(M, Dl, D2, g.b);
        if constexpr (G::n > 2) grp_finish<G::K2, GN>(M, Dl, D2, g.c);
        __builtin_amdgcn_sched_barrier(0);
        factor_pipe<GN>(M, Dl, D2, Lp, dj, dj2, yl, y2, gn);
    }
}
__device__ __forceinline__ void factor_pipelined(RegMat& M, float& Dl, float& D2, float* Lp, int dj, int dj2, float& yl,
                                                 float& y2) {
    GSteps<0> g;
    group_front<0>(M, g, Lp, dj, dj2, yl, y2);
    factor_pipe<0>(M, Dl, D2, Lp, dj, dj2, yl, y2, g);
}

}  // namespace regla
