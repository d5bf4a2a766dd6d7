// he_physics.hip -- articulated SMPL-humanoid step for gfx950 (replaces
// gym.simulate x control_freq_inv, puffer_phc/envs/humanoid_phc.py:131-134).
//
// Mapping: one environment per 64-lane workgroup (= one wave), all substeps of a policy step in
// one launch; HBM sees one coalesced read of the env's root/dof/target rows and one write of the
// root/dof/rigid-body/contact/dof-force rows.
//   * tree kinematics / RNEA / CRBA inputs: lane = body or dof, spatial quantities in LDS;
//   * joint-space algebra (75x75 mass matrix, sparse LTDL, triangular solves): register-resident,
//     lane j owns column j, fully unrolled over the static SMPL dof tree (he_regla.h);
//   * contact rows: lane = row, each lane back-substitutes its own J^T row in registers against a
//     packed copy of L read by LDS broadcast; Delassus rows by lane = column;
//   * PGS: residuals and impulses in registers, one conflict-free LDS column read per row update.
// A workgroup is a single wave, so LDS hand-offs between phases need program order only (LDS
// executes a wave's instructions in order); no s_barrier is issued.
//
// Algorithm (fp64 reference oracle/he_oracle_physics.c):
//   FK -> spatial axes S about the root origin -> RNEA bias -> CRBA (+armature) -> implicit PD
//   -> sparse LTDL -> free velocity -> ground/self contacts -> Z = L^-T J^T, A = Z^T D^-1 Z
//   -> PGS -> velocity update -> damping / clamps -> semi-implicit integration.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/humanoid_engine.h"
#include "he_kernels.h"
#include "he_math.h"
#include "he_regla.h"
#include "he_smpl_topo.h"
#include "he_topo.h"

namespace {

constexpr int NB = HE_NUM_BODIES;
constexpr int ND = HE_NUM_DOF;
constexpr int NG = HE_NUM_GEN;
constexpr int MAXC = HE_MAX_CONTACTS;  // contact slots (points, joint limits)
constexpr int MAXR = HE_MAX_ROWS;      // solver rows, one per lane (patch friction, oracle build_rows)
constexpr int W = 64;
static_assert(MAXR <= W - 1, "solver rows must fit one per lane");
constexpr int kTgsMaxIt = 16;  // TGS position iterations per physics step (he_simulate checks; oracle TGS_MAXIT)
constexpr int kTgsBiasEvery = 2;  // TGS: the bias re-evaluated every second iteration (oracle g_bias_every)
static_assert(MAXC < W, "one slot per lane in the row-layout pass");
static_assert(smpl::kNG == NG && smpl::kNB == NB, "generated topology mismatch");

struct BodyTopo {
    int8_t depth[NB];
    int8_t chain[NB][9];
    int8_t dof0[NB];
    uint32_t anc_mask[NB];
    uint32_t sub_mask[NB];
    float local_pos[NB][3];  // joint offsets (model), read along every FK chain walk
    uint32_t jump4[NB];      // byte k: 2^k-th ancestor of body b (0xFF: none), for pointer jumping
    int16_t pack_start[NG];  // packed-row offset of dof i (smpl::kPackStart)
    int8_t dof_depth[NG];    // depth of dof i in the dof tree (smpl::kDofNanc - 1)
    int8_t cbody[W];         // corner lanes: the box body of lane 24 + 8k + c (PhysTopo::corner_body)
};

struct Lds {
    float q[ND], tgt[ND];
    float u0[NG], uf[NG], rhs[NG], coef[NG], sDinv[NG];
    float yh[NG];  // D^-1/2 L^-T (dt rhs): the free motion's share of the one L^-1 sweep
    float ql[NB][4], qw[NB][4];
    float pw[NB][3];  // body origins RELATIVE to the root origin o (world axes): every spatial quantity
                      // is taken about o, and fp32 keeps ~1e-7 m of them however far o is from the
                      // world origin (world = o + pw only where a world position is needed)
    float S[NG][6], IS[NG][6];
    float V[NB][6], F[NB][6];
    alignas(16) float Acc[NB][6];  // contact phase: the bodies' bounding spheres (bsph) instead
    float Ib[NB][10], Ic[NB][10];  // m, h(3), I(xx yy zz xy xz yz)
    alignas(16) float Lp[smpl::kNpack + 4];  // packed unit-lower factor L (row K: ancestors in chain
                                             // order); Lp[kNpack] is the elimination's store sink
    float cx[MAXC][3], cn[MAXC][3], cgap[MAXC];  // slot: point about o (a joint limit: its row), normal, gap
    int cbb[MAXC];                                // slot: body0 | (body1 + 2) << 8
    float lam[W];  // impulses of the last solve (lane = row): the warm-start cache and the forces
    float cf[NB][3];
    float dforce[ND];
    float root_pos[3], root_q[4];
    float qloc[NB][4];  // each joint's local rotation exp(q_b), from the kinematics (reused by integrate)
    int nc, nterr;                 // contact slots, of which limits + terrain (slots [0, nterr))
    int nlim;                      // joint-limit slots [0, nlim) (one row each: rows [0, nlim))
    uint32_t limmask;              // bodies whose joint-angle limit row is emitted this substep
    int ncand;                     // contacts generated (dropped = ncand - nc), last substep
    alignas(8) int imbook[14];     // fused imitation: the env's bookkeeping + motion metadata (ImitBook)
    unsigned long long sch_t0;     // dispatch order: the workgroup's start cycle (PhysArgs.cost)
    int sch_e;                     // this workgroup's env (PhysArgs.order; no register held through the substeps)
    int ckey[MAXC];                // 16-bit key of each slot's normal row (include/humanoid_engine.h)
    int wckey[W];                  // the previous solve's row keys (its impulses: lam)
    int nwc;                       // rows cached in wckey / lam
    int8_t tbase[NB], tcnt[NB];    // body b's terrain contacts: slots tbase[b] .. + tcnt[b]
    int8_t srow0[MAXC];            // first solver row of each slot
    int8_t rslot[W], rkind[W];     // solver row -> its slot, its kind (0 normal / limit, 1 2 tangential, 3 torsional)
    BodyTopo T;
};

// wave priority: s_setprio 3 over the serial chains (PGS rows, the elimination, the L^-T sweeps;
// +2.8 % A/B, r01; the midpoint's L^-1 and L^-T sweeps, -1.2 % physics launch A/B, r04) against the
// partner wave's throughput phases, 0 elsewhere
constexpr int kPrioSerial = 3;
constexpr int kPrioDefault = 0;

// wave-level ordering point: one wave per workgroup, LDS executes its instructions in order, so
// only the compiler must not move memory operations across phase boundaries
HE_DEV void sync() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

HE_DEV int dof_body(int i) { return i < 6 ? 0 : (i - 6) / 3 + 1; }

// optional per-phase cycle stamps (diagnostic: PhysArgs.stamps != null), lane 0 accumulates
// s_memtime deltas per phase into stamps[block * HE_STAMP_SLOTS + phase] with a no-return vector
// atomic add (a load-add-store would put one global round trip into every phase it opens)
#ifndef HE_PHASE_STAMPS
#define HE_PHASE_STAMPS 0  // diagnostic twin library only (build.py PHASES_LIB)
#endif
#if !HE_PHASE_STAMPS
#define STAMP(id) \
    do {          \
    } while (0)
#else
#define STAMP(id)                                                             \
    do {                                                                      \
        if (stamps && lane == 0) {                                            \
            unsigned long long _t = __builtin_readcyclecounter();             \
            __hip_atomic_fetch_add(stamps + (id), _t - t_prev, __ATOMIC_RELAXED, \
                                   __HIP_MEMORY_SCOPE_AGENT);                 \
            t_prev = _t;                                                      \
        }                                                                     \
    } while (0)
#endif

// spatial inertia (m, h, I6) applied to V=(w, v): n = I w + h x v ; f = m v - h x w
HE_DEV void si_apply(const float* I, const float* V, float* F) {
    f3 h = f3{I[1], I[2], I[3]};
    f3 w = f3{V[0], V[1], V[2]}, v = f3{V[3], V[4], V[5]};
    f3 hv = cross3(h, v), hw = cross3(h, w);
    F[0] = I[4] * w.x + I[7] * w.y + I[8] * w.z + hv.x;
    F[1] = I[7] * w.x + I[5] * w.y + I[9] * w.z + hv.y;
    F[2] = I[8] * w.x + I[9] * w.y + I[6] * w.z + hv.z;
    F[3] = I[0] * v.x - hw.x;
    F[4] = I[0] * v.y - hw.y;
    F[5] = I[0] * v.z - hw.z;
}
HE_DEV float dot6(const float* a, const float* b) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}
// motion cross V x Sm
HE_DEV void crm(const float* V, const float* S, float* O) {
    f3 w = f3{V[0], V[1], V[2]}, v = f3{V[3], V[4], V[5]};
    f3 sw = f3{S[0], S[1], S[2]}, sv = f3{S[3], S[4], S[5]};
    f3 a = cross3(w, sw), b = cross3(w, sv) + cross3(v, sw);
    O[0] = a.x; O[1] = a.y; O[2] = a.z; O[3] = b.x; O[4] = b.y; O[5] = b.z;
}
// force cross V x* F
HE_DEV void crf(const float* V, const float* Fm, float* O) {
    f3 w = f3{V[0], V[1], V[2]}, v = f3{V[3], V[4], V[5]};
    f3 n = f3{Fm[0], Fm[1], Fm[2]}, f = f3{Fm[3], Fm[4], Fm[5]};
    f3 a = cross3(w, n) + cross3(v, f), b = cross3(w, f);
    O[0] = a.x; O[1] = a.y; O[2] = a.z; O[3] = b.x; O[4] = b.y; O[5] = b.z;
}


// rotation-vector exponential / logarithm for the physics kernel, short instruction sequences (the
// integration runs them in every TGS position iteration): v_sqrt_f32 and v_rcp_f32 (1 ulp), sin / cos
// of the half angle by their Taylor series up to x^9 / x^10 (|x| <= 1: error < 3e-8, below fp32
// rounding; a step turning a joint by more than 2 rad takes ocml's sincosf), atan on [0, 1] by
// Abramowitz-Stegun 4.4.49 (|error| <= 1e-8). The fp64 oracle's tolerance covers them. The imitation
// kernel keeps he_math.h's forms, which follow torch's rounding.
// a polynomial's second coefficient materialised where it is used (the FMAs take the others as
// literals): left to the compiler, it is hoisted out of the TGS iterations into a register held
// through them, and that register pushes the loop's long-lived state into scratch
template <uint32_t BITS>
HE_DEV float here(void) {
    float r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "n"(BITS));
    return r;
}
HE_DEV void half_sincos(float x, float& sn, float& cs) {
    if (__builtin_expect(x > 1.0f, 0)) {
        sincosf(x, &sn, &cs);
        return;
    }
    const float x2 = x * x;
    float ps = fmaf(x2, 2.75573192e-6f, here<0xb9500d01u>());  // -1.98412698e-4
    ps = fmaf(x2, ps, 8.33333333e-3f);
    ps = fmaf(x2, ps, -1.66666667e-1f);
    sn = fmaf(x * x2, ps, x);
    float pc = fmaf(x2, -2.75573192e-7f, here<0x37d00d01u>());  // 2.48015873e-5
    pc = fmaf(x2, pc, -1.38888889e-3f);
    pc = fmaf(x2, pc, 4.16666667e-2f);
    pc = fmaf(x2, pc, -0.5f);
    cs = fmaf(x2, pc, 1.0f);
}
HE_DEV float atan01(float t) {  // t in [0, 1]
    const float t2 = t * t;
    float p = fmaf(t2, 0.0028662257f, here<0xbc846e02u>());  // -0.0161657367
    p = fmaf(t2, p, 0.0429096138f);
    p = fmaf(t2, p, -0.0752896400f);
    p = fmaf(t2, p, 0.1065626393f);
    p = fmaf(t2, p, -0.1420889944f);
    p = fmaf(t2, p, 0.1999355085f);
    p = fmaf(t2, p, -0.3333314528f);
    return fmaf(t * t2, p, t);
}
HE_DEV f4 pqexp(f3 v) {
    const float th = __builtin_amdgcn_sqrtf(dot3(v, v));
    if (th < 1e-8f) return qnormalize(f4{0.5f * v.x, 0.5f * v.y, 0.5f * v.z, 1.f});
    float sh, ch;
    half_sincos(0.5f * th, sh, ch);
    const float s = sh * __builtin_amdgcn_rcpf(th);
    return f4{v.x * s, v.y * s, v.z * s, ch};
}
HE_DEV f3 pqlog(f4 q) {
    if (q.w < 0.f) q = qneg(q);
    const float s = __builtin_amdgcn_sqrtf(q.x * q.x + q.y * q.y + q.z * q.z);
    if (s < 1e-8f) return f3{2.f * q.x, 2.f * q.y, 2.f * q.z};
    // atan2(s, w) on the first quadrant (s > 0, w >= 0): the smaller over the larger, then pi / 2 - a
    const float lo = fminf(s, q.w), hi = fmaxf(s, q.w);
    const float a = atan01(lo * __builtin_amdgcn_rcpf(hi));
    const float ang = s > q.w ? 1.57079632679f - a : a;
    const float k = 2.f * ang * __builtin_amdgcn_rcpf(s);
    return f3{q.x * k, q.y * k, q.z * k};
}

// Joint-angle limit of joint b (oracle/he_oracle_physics.c angle_row): the exp-map coordinate
// wraps at |q_b| = pi, so the MJCF's +-180 / +-720 deg ranges hold the rotation angle at
// pi - kLimitGuard; the speculative row is emitted within limit_margin + dt * (closing rate).
constexpr float kLimitGuard = 0.02f;
HE_DEV bool angle_row(f3 th, f3 u, const he_sim_params& p, float& gap, f3& dir) {
    const float t = __builtin_amdgcn_sqrtf(dot3(th, th));
    dir = th * __builtin_amdgcn_rcpf(fmaxf(t, 1e-30f));
    gap = (3.14159265358979f - kLimitGuard) - t;
    const float closing = dot3(dir, u);
    return t >= 1e-6f && gap < p.limit_margin + p.dt * fmaxf(closing, 0.f);
}

// the bodies' bounding spheres of the self-collision cull, in the RNEA acceleration scratch (dead
// from the midpoint bias until the next substep's kinematics)
HE_DEV float4* bsph(Lds& L) { return reinterpret_cast<float4*>(&L.Acc[0][0]); }
static_assert(sizeof(float4) * NB <= sizeof(float) * 6 * NB, "bounding spheres fit the Acc scratch");
// Backstop when the limit rows lose (oracle/he_oracle_physics.c limit_clamp): a limit against a
// deep self contact has no solution, and a joint near 100 rad/s can cross the margin in one
// substep. nq = exp(q_old) (x) exp(dt w) before the log (exp(q_old) has w >= 0: the kinematics'
// and this function's qloc): its scalar part is negative when the rotation went past pi this
// substep, and the log then comes back on the far side with the axis flipped, which would reverse
// the joint's PD error and spin it. The angle is continued past pi instead, then held at
// pi - kLimitGuard / 2 on the joint's side with the outward rate q^ . w removed. Returns whether it
// acted (nv and w changed).
HE_DEV bool limit_clamp(f4 nq, f3& nv, float (&w)[3]) {
    constexpr float kTwoPi = 6.28318530717959f;
    constexpr float cap = 3.14159265358979f - 0.5f * kLimitGuard;
    constexpr float kWcap = 0.00499997917f;  // cos(cap / 2)
    if (nq.w >= kWcap) return false;         // inside the cap, not crossed: the common case
    const float t0 = sqrtf(dot3(nv, nv));
    if (!(t0 >= 1e-12f)) return false;
    f3 dir = nv * (1.0f / t0);
    float t = t0;
    if (nq.w < 0.f) {
        t = kTwoPi - t0;
        dir = dir * -1.f;
    }
    if (t <= cap) return false;
    nv = dir * cap;
    const float out = dir.x * w[0] + dir.y * w[1] + dir.z * w[2];
    if (out > 0.f) { w[0] -= out * dir.x; w[1] -= out * dir.y; w[2] -= out * dir.z; }
    return true;
}

// Which joints emit their limit row in the next substep, from joint b's exp map th and velocity u
// (lane = body b; every lane calls, the root and lanes >= NB with on = false), read by the drive
// terms (a joint on its limit cannot give way). Evaluated where q and u are set -- the state load,
// then each integration but the last; the contact phase re-evaluates the rows themselves from the
// same L.q / L.u0 (bit-identical inputs, the same decision).
HE_DEV void limit_detect(Lds& L, int lane, bool joint, f3 th, f3 u, const he_sim_params& sp) {
    float lg = 0.f;
    f3 ld = f3{0.f, 0.f, 0.f};
    const bool on = joint && angle_row(th, u, sp, lg, ld);
    const uint64_t bm = __ballot(on);
    if (lane == 0) L.limmask = (uint32_t)bm;
}

// terrain constants of the env, read once per contact phase (slope normal, step field)
struct Terrain {
    int kind;
    float sn, cs, step_h, step_l;
};
HE_DEV Terrain terrain_of(const he_sim_params& p, int kind) {
    Terrain t{kind, 0.f, 1.f, p.step_height, p.step_length};
    if (kind == 1) { t.sn = sinf(p.terrain_slope); t.cs = cosf(p.terrain_slope); }
    return t;
}
HE_DEV float terrain_dist(const Terrain& t, f3 x, f3& n) {
    if (t.kind == 1) {
        n = f3{-t.sn, 0.f, t.cs};
        return dot3(n, x);
    }
    n = f3{0.f, 0.f, 1.f};
    if (t.kind == 2) {
        float h = x.x > 0.f ? t.step_h * floorf(x.x / t.step_l) : 0.f;
        return x.z - h;
    }
    return x.z;
}

// closest points between segments p1q1 and p2q2 (Ericson, RTCD 5.1.9), branch-free: every case
// (both degenerate, one degenerate, general with its two t-clamps) is formed and selected, so a
// wave of mixed sphere / capsule pairs runs one path
HE_DEV void seg_seg(f3 p1, f3 q1, f3 p2, f3 q2, f3& c1, f3& c2) {
    const f3 d1 = q1 - p1, d2 = q2 - p2, r = p1 - p2;
    const float a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    const float eps = 1e-12f;
    // divisions as v_rcp_f32 products (1 ulp; the fp64 oracle's tolerance covers it)
    const float ia = __builtin_amdgcn_rcpf(a), ie = __builtin_amdgcn_rcpf(e);
    const float c = dot3(d1, r), b = dot3(d1, d2), den = a * e - b * b;
    const float sg = den > eps ? __builtin_amdgcn_fmed3f((b * f - c * e) * __builtin_amdgcn_rcpf(den), 0.f, 1.f) : 0.f;
    const float tg = (b * sg + f) * ie;
    const float s_lo = __builtin_amdgcn_fmed3f(-c * ia, 0.f, 1.f);       // t clamped to 0 (and e degenerate)
    const float s_hi = __builtin_amdgcn_fmed3f((b - c) * ia, 0.f, 1.f);  // t clamped to 1
    float s = tg < 0.f ? s_lo : (tg > 1.f ? s_hi : sg);
    float t = tg < 0.f ? 0.f : (tg > 1.f ? 1.f : tg);
    const bool adeg = a <= eps, edeg = e <= eps;
    s = edeg ? s_lo : s;
    t = edeg ? 0.f : t;
    s = adeg ? 0.f : s;
    t = adeg ? (edeg ? 0.f : __builtin_amdgcn_fmed3f(f * ie, 0.f, 1.f)) : t;
    c1 = p1 + d1 * s;
    c2 = p2 + d2 * t;
}

HE_DEV void friction_basis(f3 n, f3& t1, f3& t2) {
    f3 a = fabsf(n.x) > 0.9f ? f3{0.f, 1.f, 0.f} : f3{1.f, 0.f, 0.f};
    float d = dot3(a, n);
    t1 = a - n * d;
    t1 = t1 * (1.0f / norm3(t1));
    t2 = cross3(n, t1);
}

// OR over the wave as a wave-uniform value: quad and row DPP mirrors, then the 16- and 32-lane
// permlane swaps (no LDS crossbar round trips)
HE_DEV uint32_t wave_or(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
    x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false);  // row_mirror
    const auto r16 = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    x = r16[0] | r16[1];
    const auto r32 = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    x = r32[0] | r32[1];
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}

// wave-wide exclusive prefix count of `flag` (uint64 ballot)
HE_DEV int wave_prefix(bool flag, int lane, int& total) {
    uint64_t m = __ballot(flag);
    total = __popcll(m);
    uint64_t below = lane == 0 ? 0ull : (m & ((~0ull) >> (64 - lane)));
    return __popcll(below);
}

// the value of lane ^ S (S < 32): ds_swizzle in bitmask mode (and 0x1F, xor S)
template <int S>
HE_DEV float swizzle_xor(float v) {
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x1F | (S << 10)));
}
HE_DEV void store_contact(Lds& L, int slot, int b0, int b1, f3 x, f3 n, float gap, int key) {
    L.cbb[slot] = b0 | ((b1 + 2) << 8);
    L.cx[slot][0] = x.x; L.cx[slot][1] = x.y; L.cx[slot][2] = x.z;
    L.cn[slot][0] = n.x; L.cn[slot][1] = n.y; L.cn[slot][2] = n.z;
    L.cgap[slot] = gap;
    L.ckey[slot] = key;
}
// 16-bit row keys (include/humanoid_engine.h cache layout)
HE_DEV int row_key(int b0, int b1, int sub, int kind) { return b0 | ((b1 + 2) << 5) | (sub << 10) | (kind << 14); }

// ordered multiply / multiply-add (volatile asm keeps program order against the surrounding LDS
// reads, so the unrolled sweeps do not hoist every load ahead of the arithmetic)
template <class T>
HE_DEV const T* opaque(const T* p) {  // same address through an opaque offset: pins dependent loads
    int off = 0;
    asm volatile("" : "+v"(off));
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(p) + off);
}

// Delassus operator on the matrix cores: A = Zh Zh^T as four 32x32 tiles of
// v_mfma_f32_32x32x2_f32 (exact f32, k-ordered fma chain), K = live dofs two at a time. Lane r
// holds row r of Zh; one v_permlane32_swap per dof pair turns (z[k], z[k+1]) into the A/B operand
// of rows 0-31 (p0) and of rows 32-63 (p1). A second round of swaps moves the C tiles
// (col = lane & 31, row = (v & 3) + 8 (v >> 2) + 4 (lane >> 5)) into "lane c holds column c".
constexpr int NGRP = (NG + 3) / 4;  // dof groups of four
typedef float f32x16 __attribute__((ext_vector_type(16)));
HE_DEV void swap32(float& a, float& b) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
HE_DEV void swap16(float& a, float& b) {  // odd 16-lane rows of a <-> even rows of b
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
template <int CTRL>
HE_DEV float dpp(float x) { return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false)); }

// One butterfly stage of a wave reduce-scatter below 16 lanes: the partner (DPP pattern CTRL, an
// involution flipping lane bit B) gets the half this lane drops; lanes with bit B keep the upper
// half. H = values kept.
template <int H, int CTRL, uint64_t BITMASK>
HE_DEV void rs_dpp(float* v) {
    const bool up = regla::lanes<BITMASK>();
#pragma unroll
    for (int j = 0; j < H; ++j) {
        const float send = up ? v[j] : v[j + H];
        const float keep = up ? v[j + H] : v[j];
        v[j] = keep + dpp<CTRL>(send);
    }
}

// Reduce-scatter of N = 64 or 16 per-lane values: returns sum over all lanes of v[idx(lane)], with
// idx = lane (N = 64) or lane >> 2 (N = 16). Pairings by lane-bit flips 32, 16 (permlane swaps),
// 15 (row mirror), 7 (half-row mirror), 2, 1 (quad perms): independent, so every lane's result
// covers all 64 lanes once; 63 exchanges + 63 adds for 64 values (vs 6 x 64 for all-reduce).
template <int N>
HE_DEV float reduce_scatter(float (&v)[N]) {
#pragma unroll
    for (int j = 0; j < N / 2; ++j) { swap32(v[j], v[j + N / 2]); v[j] += v[j + N / 2]; }
#pragma unroll
    for (int j = 0; j < N / 4; ++j) { swap16(v[j], v[j + N / 4]); v[j] += v[j + N / 4]; }
    rs_dpp<N / 8, 0x140, 0xFF00FF00FF00FF00ull>(v);  // row_mirror: lane ^ 15
    rs_dpp<N / 16, 0x141, 0xF0F0F0F0F0F0F0F0ull>(v);  // row_half_mirror: lane ^ 7
    if constexpr (N == 64) {
        rs_dpp<2, 0x4E, 0xCCCCCCCCCCCCCCCCull>(v);  // quad_perm [2,3,0,1]: lane ^ 2
        rs_dpp<1, 0xB1, 0xAAAAAAAAAAAAAAAAull>(v);  // quad_perm [1,0,3,2]: lane ^ 1
    } else {
        v[0] += dpp<0x4E>(v[0]);  // the 4 lanes of a quad hold the same index: all-reduce them
        v[0] += dpp<0xB1>(v[0]);
    }
    return v[0];
}
// Zh^T x into lane = dof (lane i: sum over rows r of z_r[i] x_r; lanes < 11 also dof 64 + lane in e2): the
// same butterfly as reduce_scatter with the products formed as the first stage consumes them, so at
// most 32 + 8 of them are live at once (the TGS iterations run it beside the rows' Zh and columns)
// zh_r . y with y_i broadcast from lane i (yl: dofs 0..63, y2: dofs 64..74 on lanes 0..10): the
// readlanes in blocks of four SGPRs (one hazard nop per block), the products on the register pairs
// (v_pk_fma: half the VALU), the four partial sums of the scalar form (dof i into sum i mod 4),
// so the result is that form's to the bit
HE_DEV float zdot_lanes(const regla::ZVec& z, float yl, float y2) {
    using regla::f2v;
    f2v a = f2v{0.f, 0.f}, b = f2v{0.f, 0.f};
    regla::static_for<0, NG, 4>([&](auto ic) {
        constexpr int i0 = decltype(ic)::value;
        float sv[4];
        if constexpr (i0 < 64) regla::rdlane4<i0>(yl, sv);
        else regla::rdlane4<i0 - 64>(y2, sv);
        a = __builtin_elementwise_fma(z.p[i0 >> 1], f2v{sv[0], sv[1]}, a);
        if constexpr (i0 + 3 < NG) b = __builtin_elementwise_fma(z.p[(i0 >> 1) + 1], f2v{sv[2], sv[3]}, b);
        else if constexpr (i0 + 2 < NG) b.x = fmaf(ZV(z, i0 + 2), sv[2], b.x);
    });
    return (a.x + a.y) + (b.x + b.y);
}
// The products and the first two stages' sums run on the register pairs (v_pk_mul / v_pk_add: half the
// VALU of the scalar forms, the same IEEE results)
HE_DEV void reduce_scatter_z(const regla::ZVec& z, float x, int lane, float& e1, float& e2) {
    using regla::f2v;
    const f2v xx = f2v{x, x};
    float v[32];
#pragma unroll
    for (int j = 0; j < 32; j += 2) {
        const f2v pa = z.p[j >> 1] * xx, pb = z.p[(j + 32) >> 1] * xx;
        float a0 = pa.x, b0 = pb.x, a1 = pa.y, b1 = pb.y;
        swap32(a0, b0);
        swap32(a1, b1);
        const f2v s = f2v{a0, a1} + f2v{b0, b1};
        v[j] = s.x;
        v[j + 1] = s.y;
    }
#pragma unroll
    for (int j = 0; j < 16; j += 2) {
        swap16(v[j], v[j + 16]);
        swap16(v[j + 1], v[j + 17]);
        const f2v s = f2v{v[j], v[j + 1]} + f2v{v[j + 16], v[j + 17]};
        v[j] = s.x;
        v[j + 1] = s.y;
    }
    rs_dpp<8, 0x140, 0xFF00FF00FF00FF00ull>(v);
    rs_dpp<4, 0x141, 0xF0F0F0F0F0F0F0F0ull>(v);
    rs_dpp<2, 0x4E, 0xCCCCCCCCCCCCCCCCull>(v);
    rs_dpp<1, 0xB1, 0xAAAAAAAAAAAAAAAAull>(v);
    e1 = v[0];
    float w[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float a = 64 + j < NG ? ZV(z, 64 + j < NG ? 64 + j : 0) * x : 0.f;
        float b = 72 + j < NG ? ZV(z, 72 + j < NG ? 72 + j : 0) * x : 0.f;
        swap32(a, b);
        w[j] = a + b;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) { swap16(w[j], w[j + 4]); w[j] += w[j + 4]; }
    rs_dpp<2, 0x140, 0xFF00FF00FF00FF00ull>(w);
    rs_dpp<1, 0x141, 0xF0F0F0F0F0F0F0F0ull>(w);
    w[0] += dpp<0x4E>(w[0]);
    w[0] += dpp<0xB1>(w[0]);
    e2 = __shfl(w[0], 4 * (lane & 15), W);
}
// The rows' support inside the root and the two legs (bodies 0..8: dofs 0..29, the DFS prefix; a body
// standing or walking on its feet): Zh is zero past dof 29, so the iterations' products run over the
// first KZ = 32 dofs (dofs 30, 31 exact zeros) with Zh's other 44 registers dead.
#ifndef HE_TGS_LEGS  // A/B only: 0 runs every env's iterations over all 75 dofs
#define HE_TGS_LEGS 1
#endif
#ifndef HE_TGS_LEGS_ROWS  // A/B only: 0 runs the rows' once-per-step dot products over all 75 dofs
#define HE_TGS_LEGS_ROWS 1
#endif
constexpr uint32_t kLegBodies = 0x1FFu;
constexpr int KZ = 32;
static_assert(smpl::kNB > 9, "the leg prefix is bodies 0..8");
// zdot_lanes over dofs 0..KZ-1: bit for bit the full form (its dropped terms are fma(0, y, s) = s)
HE_DEV float zdot_lanes_legs(const regla::ZVec& z, float yl) {
    using regla::f2v;
    f2v a = f2v{0.f, 0.f}, b = f2v{0.f, 0.f};
    regla::static_for<0, KZ, 4>([&](auto ic) {
        constexpr int i0 = decltype(ic)::value;
        float sv[4];
        regla::rdlane4<i0>(yl, sv);
        a = __builtin_elementwise_fma(z.p[i0 >> 1], f2v{sv[0], sv[1]}, a);
        b = __builtin_elementwise_fma(z.p[(i0 >> 1) + 1], f2v{sv[2], sv[3]}, b);
    });
    return (a.x + a.y) + (b.x + b.y);
}
// Zh^T x over dofs 0..KZ-1 into lane = dof: the butterfly's stages inside each 32-lane half (lane bits
// 4 .. 0: the 32 values to one per lane), then the two halves' partial sums added (lane bit 5). Lanes
// >= KZ return 0 (e2 = 0: no dof past 63 is on the support). The same sum as reduce_scatter_z's in
// another association order.
HE_DEV float reduce_scatter_z_legs(const regla::ZVec& z, float x) {
    using regla::f2v;
    const f2v xx = f2v{x, x};
    float v[KZ];
#pragma unroll
    for (int j = 0; j < KZ / 2; j += 2) {
        const f2v pa = z.p[j >> 1] * xx, pb = z.p[(j + KZ / 2) >> 1] * xx;
        float a0 = pa.x, b0 = pb.x, a1 = pa.y, b1 = pb.y;
        swap16(a0, b0);
        swap16(a1, b1);
        const f2v s = f2v{a0, a1} + f2v{b0, b1};
        v[j] = s.x;
        v[j + 1] = s.y;
    }
    rs_dpp<8, 0x140, 0xFF00FF00FF00FF00ull>(v);
    rs_dpp<4, 0x141, 0xF0F0F0F0F0F0F0F0ull>(v);
    rs_dpp<2, 0x4E, 0xCCCCCCCCCCCCCCCCull>(v);
    rs_dpp<1, 0xB1, 0xAAAAAAAAAAAAAAAAull>(v);
    float a = v[0], b = v[0];
    swap32(a, b);  // a: lanes < 32 their own half's sum, b: the other half's (lanes >= 32: swapped roles)
    const float e = a + b;
    return regla::lanes<0xFFFFFFFFull>() ? e : 0.f;
}
// at most 32 rows (<= 10 contacts): only the rows-0-31 x columns-0-31 tile is needed (one MFMA per
// dof pair instead of four); rows >= 32 of acol are never read then
HE_DEV void delassus_mfma32(const regla::ZVec& z, float (&acol)[MAXR], uint32_t live) {
    f32x16 t00 = {};
#pragma unroll
    for (int g = 0; g < NGRP; ++g) {
        if ((live >> g) & 1u) {
#pragma unroll
            for (int h = 0; h < 4; h += 2) {
                const int k0 = 4 * g + h;
                if (k0 < NG) {
                    float p0 = ZV(z, k0), p1 = k0 + 1 < NG ? ZV(z, k0 + 1 < NG ? k0 + 1 : 0) : 0.f;
                    swap32(p0, p1);
                    t00 = __builtin_amdgcn_mfma_f32_32x32x2f32(p0, p0, t00, 0, 0, 0);
                }
            }
        }
    }
    const f32x16 zero = {};
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const int r = (v & 3) + 8 * (v >> 2);
        float a = t00[v], b = zero[v];
        swap32(a, b);  // a: A[r][lane], b: A[r + 4][lane] (lanes >= 32: zero)
        acol[r] = a;
        acol[r + 4] = b;
        if (32 + r < MAXR) acol[32 + r < MAXR ? 32 + r : 0] = 0.f;
        if (36 + r < MAXR) acol[36 + r < MAXR ? 36 + r : 0] = 0.f;
    }
}
// 33-48 rows (11-16 contacts): 16x16x4 tiles over three row blocks instead of four 32x32 tiles
// (9 x 32 cycles per four dofs instead of 8 x 64). Operands: a 4x4 transpose of (register,
// 16-lane group) by two permlane32 and two permlane16 swaps turns z[k0..k0+3] into the A/B
// operand of each row block; results: the same transpose moves each tile's 4 row quads into the
// column's lane group (lane c holds A[r][c]).
typedef float f32x4 __attribute__((ext_vector_type(4)));
HE_DEV void xpose4(float (&r)[4]) {  // r[i] <- (group g: r[g] of group i)
    swap32(r[0], r[2]);
    swap32(r[1], r[3]);
    swap16(r[0], r[1]);
    swap16(r[2], r[3]);
}
HE_DEV void delassus_mfma48(const regla::ZVec& z, float (&acol)[MAXR], uint32_t live) {
    f32x4 c[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) c[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < NGRP; ++g) {
        if ((live >> g) & 1u) {
            float r[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) r[k] = 4 * g + k < NG ? ZV(z, 4 * g + k < NG ? 4 * g + k : 0) : 0.f;
            xpose4(r);
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 3; ++j) c[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(r[i], r[j], c[i][j], 0, 0, 0);
        }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            float x[4] = {c[i][0][v], c[i][1][v], c[i][2][v], 0.f};
            xpose4(x);  // x[g] on lane c: A[16 i + 4 g + v][c]
#pragma unroll
            for (int g = 0; g < 4; ++g) acol[16 * i + 4 * g + v] = x[g];
        }
#pragma unroll
    for (int r = 48; r < MAXR; ++r) acol[r] = 0.f;
}
HE_DEV void delassus_mfma(const regla::ZVec& z, float (&acol)[MAXR], uint32_t live) {
    f32x16 t00 = {}, t01 = {}, t10 = {}, t11 = {};
#pragma unroll
    for (int g = 0; g < NGRP; ++g) {
        if ((live >> g) & 1u) {
#pragma unroll
            for (int h = 0; h < 4; h += 2) {
                const int k0 = 4 * g + h;
                if (k0 < NG) {
                    float p0 = ZV(z, k0), p1 = k0 + 1 < NG ? ZV(z, k0 + 1 < NG ? k0 + 1 : 0) : 0.f;
                    swap32(p0, p1);
                    t00 = __builtin_amdgcn_mfma_f32_32x32x2f32(p0, p0, t00, 0, 0, 0);
                    t01 = __builtin_amdgcn_mfma_f32_32x32x2f32(p0, p1, t01, 0, 0, 0);
                    t10 = __builtin_amdgcn_mfma_f32_32x32x2f32(p1, p0, t10, 0, 0, 0);
                    t11 = __builtin_amdgcn_mfma_f32_32x32x2f32(p1, p1, t11, 0, 0, 0);
                }
            }
        }
    }
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const int r = (v & 3) + 8 * (v >> 2);
        float a = t00[v], b = t01[v], c = t10[v], d = t11[v];
        swap32(a, b);  // a: A[r][lane], b: A[r + 4][lane]
        swap32(c, d);  // c: A[32 + r][lane], d: A[36 + r][lane]
        acol[r] = a;
        acol[r + 4] = b;
        if (32 + r < MAXR) acol[32 + r < MAXR ? 32 + r : 0] = c;
        if (36 + r < MAXR) acol[36 + r < MAXR ? 36 + r : 0] = d;
    }
}

// One Gauss-Seidel sweep, branch-free: every row up to a compile-time class bound N (16, 32, 48,
// 63) by the row count, with no per-row row-count branch (a row-count exit every 4 rows); rows nr..N-1 are empty rows (zero columns and
// bound weights in every lane, zero cd and bounds in their own lanes: a +-0 change).
template <int R, int N, int M = MAXR>
HE_DEV void pgs_sweep_fix(regla::f2v& ch, float& dvec, float& lo, const regla::f2v (&ak)[M], int nr) {
    if constexpr (R < N) {
        if constexpr (R > 0 && R % 4 == 0) {  // a row-count exit every 4 rows
            if (R >= nr) return;
        }
        const float d = regla::rdlane(__builtin_amdgcn_fmed3f(ch.x, lo, ch.y), R);
        ch = __builtin_elementwise_fma(ak[R], regla::f2v{d, d}, ch);
        lo = fmaf(-ak[R].y, d, lo);
        dvec = regla::wrlane<R>(d, dvec);
        pgs_sweep_fix<R + 1, N, M>(ch, dvec, lo, ak, nr);
    }
}

// TGS (solver_type 1): the same sweep with the friction bound weights rebuilt per row from the lane's
// patch mask (2 VALU off the dependent chain) instead of a second register per row: the scaled
// columns, the rows' Zh and the sweep state stay in registers through the position iterations'
// triangular solves, bias passes and integrations
template <int R, int N, int M>
HE_DEV void pgs_sweep_tgs(regla::f2v& ch, float& dvec, float& lo, const float (&ap)[M], uint32_t mlo, uint32_t mhi,
                          float muw, int nr) {
    static_assert(N <= M, "the sweep's rows within the columns held");
    if constexpr (R < N) {
        if constexpr (R > 0 && R % 4 == 0) {  // a row-count exit every 4 rows
            if (R >= nr) return;
        }
        const float d = regla::rdlane(__builtin_amdgcn_fmed3f(ch.x, lo, ch.y), R);
        const int sel = __builtin_amdgcn_sbfe((int)(R < 32 ? mlo : mhi), R & 31, 1);
        const float wr = __int_as_float(sel & __float_as_int(muw));
        // scalar FMAs: a packed pair built from ap[R] makes the compiler load ap as overlapping
        // two-float vectors, which keeps the whole column array in scratch
        ch.x = fmaf(ap[R], d, ch.x);
        ch.y = fmaf(wr, d, ch.y);
        lo = fmaf(-wr, d, lo);
        dvec = regla::wrlane<R>(d, dvec);
        pgs_sweep_tgs<R + 1, N, M>(ch, dvec, lo, ap, mlo, mhi, muw, nr);
    }
}

// CRBA straight into registers: lane j owns column j, H[i][j] = S_j . IS_i for j in chain(i)
// (compile-time lane masks), plus armature and the implicit-drive terms on the diagonal
// ---- contact-row helpers (rows phase)
// bodies touched by dof group g (4 dofs), as a mask over bodies
struct GroupBodies {
    uint32_t m[(NG + 3) / 4];
    constexpr GroupBodies() : m() {
        for (int g = 0; g < (NG + 3) / 4; ++g) {
            m[g] = 0u;
            for (int k = 0; k < 4; ++k)
                if (4 * g + k < NG) m[g] |= 1u << smpl::kDofBody[4 * g + k];
        }
    }
};
constexpr GroupBodies kGroupBodiesT{};
constexpr const uint32_t* kGroupBodies = kGroupBodiesT.m;

// joint b's data for the row Jacobian: body origin (3), its 3 joint axes (9), their free velocities (3)
HE_DEV void zrow_load(const Lds& L, int b, float (&d)[15]) {
    const Lds& Lg = *opaque(&L);
    for (int x = 0; x < 3; ++x) d[x] = Lg.pw[b][x];
    for (int c = 0; c < 3; ++c) {
        const int i = 6 + 3 * (b - 1) + c;
        for (int x = 0; x < 3; ++x) d[3 + 3 * c + x] = Lg.S[i][x];
        d[12 + c] = Lg.uf[i];
    }
}
// z = J_r^T on the matrix cores: C[i][r] = S_i . u_r with u_r = (rho, dd) of row r (lane r), as
// v_mfma_f32_32x32x2_f32 tiles over the dof blocks of 32 that hold a live body (A = S from LDS, B =
// the rows' 6-vectors redistributed by one permlane32 swap per k step). The two row tiles of a
// block are paired by v_permlane32_swap into "lane r holds z[r][i]" (ZVec); then each dof takes its
// body's sign for the row (+1 on the first contact body's chain, -1 on the second's, 0 elsewhere).
constexpr uint32_t block_bodies(int D) {
    uint32_t m = 0;
    for (int i = 32 * D; i < 32 * D + 32 && i < NG; ++i) m |= 1u << (i < 6 ? 0 : (i - 6) / 3 + 1);
    return m;
}
template <int D>
HE_DEV void zrows_block(regla::ZVec& z, uint32_t lb, const float (&b0)[3], const float (&b1)[3], const Lds& L, int l31,
                        int kh, bool rows32) {
    if constexpr (32 * D < NG) {
        if (lb & block_bodies(D)) {
            float aS[3];
            const int j = 32 * D + l31;
#pragma unroll
            for (int st = 0; st < 3; ++st) aS[st] = j < NG ? L.S[j < NG ? j : 0][2 * st + kh] : 0.f;
            f32x16 t0 = {}, t1 = {};
#pragma unroll
            for (int st = 0; st < 3; ++st) t0 = __builtin_amdgcn_mfma_f32_32x32x2f32(aS[st], b0[st], t0, 0, 0, 0);
            if (!rows32) {  // rows 32-63 exist (wave-uniform)
#pragma unroll
                for (int st = 0; st < 3; ++st) t1 = __builtin_amdgcn_mfma_f32_32x32x2f32(aS[st], b1[st], t1, 0, 0, 0);
            }
#pragma unroll
            for (int v = 0; v < 16; ++v) {
                const int i = 32 * D + (v & 3) + 8 * (v >> 2);
                float a = t0[v], b = t1[v];
                swap32(a, b);  // a: z[lane][i], b: z[lane][i + 4]
                if (i < NG) ZV(z, i < NG ? i : 0) = a;
                if (i + 4 < NG) ZV(z, i + 4 < NG ? i + 4 : 0) = b;
            }
        } else {
#pragma unroll
            for (int i = 32 * D; i < 32 * D + 32 && i < NG; ++i) ZV(z, i) = 0.f;
        }
        zrows_block<D + 1>(z, lb, b0, b1, L, l31, kh, rows32);
    }
}
HE_DEV void zrows_mfma(regla::ZVec& z, uint32_t lb, uint32_t anc0, uint32_t anc1, f3 rho, f3 dd, const Lds& L,
                       int lane, bool rows32) {
    const int l31 = lane & 31, kh = lane >> 5;
    float b0[3], b1[3];
    {
        const float u[6] = {rho.x, rho.y, rho.z, dd.x, dd.y, dd.z};
#pragma unroll
        for (int st = 0; st < 3; ++st) {
            float x = u[2 * st], y = u[2 * st + 1];
            swap32(x, y);  // x: B operand of rows 0-31, y: of rows 32-63
            b0[st] = x;
            b1[st] = y;
        }
    }
    zrows_block<0>(z, lb, b0, b1, L, l31, kh, rows32);
    float sg[NB];
#pragma unroll
    for (int B = 0; B < NB; ++B) sg[B] = (float)((anc0 >> B) & 1u) - (float)((anc1 >> B) & 1u);
#pragma unroll
    for (int i = 0; i < NG; ++i) ZV(z, i) *= sg[i < 6 ? 0 : (i - 6) / 3 + 1];
}

// z_i = S_i . (rho, dd) = a_i . ((x - p_b) x dd) for joint b's three dofs, bodies in order with
// the next live body's data read while this one is computed
template <int B>
HE_DEV void zrow_bodies(regla::ZVec& z, float (&bacc)[4], uint32_t lb, uint32_t anc0, uint32_t anc1, f3 cx, f3 dd,
                        const Lds& L, const float (&cur)[15]) {
    if constexpr (B < NB) {
        float nxt[15];
        if constexpr (B + 1 < NB) {
            if ((lb >> (B + 1)) & 1u) zrow_load(L, B + 1, nxt);
            else
                for (int x = 0; x < 15; ++x) regla::undef_reg(nxt[x]);  // never read: no zeros
        }
        constexpr int i0 = 6 + 3 * (B - 1);
        if ((lb >> B) & 1u) {
            const float sgn = (float)((anc0 >> B) & 1u) - (float)((anc1 >> B) & 1u);
            const f3 v = cross3(cx - f3{cur[0], cur[1], cur[2]}, dd) * sgn;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                ZV(z, i0 + c) = cur[3 + 3 * c] * v.x + cur[4 + 3 * c] * v.y + cur[5 + 3 * c] * v.z;
                bacc[c] = fmaf(ZV(z, i0 + c), cur[12 + c], bacc[c]);
            }
        } else {
            ZV(z, i0) = 0.f; ZV(z, i0 + 1) = 0.f; ZV(z, i0 + 2) = 0.f;
        }
        asm volatile("" : "+v"(z.p[i0 >> 1]), "+v"(z.p[(i0 + 2) >> 1]), "+v"(bacc[0]), "+v"(bacc[1]), "+v"(bacc[2]));
        zrow_bodies<B + 1>(z, bacc, lb, anc0, anc1, cx, dd, L, nxt);
    }
}
template <int I, int N = NG>
HE_DEV void scale_rows(regla::ZVec& z, float sdl, float sdl2) {
    if constexpr (I < N) {
        ZV(z, I) *= I < 64 ? regla::rdlane(sdl, I < 64 ? I : 0) : regla::rdlane(sdl2, I >= 64 ? I - 64 : 0);
        scale_rows<I + 1, N>(z, sdl, sdl2);
    }
}
// the rows' dot products over the register pairs (dof i into partial sum i mod 4) over dofs 0..N-1:
// sum_i a_r[i] u_i with u read from LDS (J_r u0), and |zh_r|^2
template <int N>
HE_DEV float zdot_lds(const regla::ZVec& z, const float* u) {
    float bacc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < N / 2; ++k) {
        const regla::f2v uk = *reinterpret_cast<const regla::f2v*>(&u[2 * k]);
        regla::f2v acc = regla::f2v{bacc[(2 * k) & 3], bacc[(2 * k + 1) & 3]};
        acc = __builtin_elementwise_fma(z.p[k], uk, acc);
        bacc[(2 * k) & 3] = acc.x;
        bacc[(2 * k + 1) & 3] = acc.y;
    }
    if constexpr (N & 1) bacc[(N - 1) & 3] = fmaf(ZV(z, N - 1), u[N - 1], bacc[(N - 1) & 3]);
    return (bacc[0] + bacc[1]) + (bacc[2] + bacc[3]);
}
template <int N>
HE_DEV float znorm2(const regla::ZVec& z) {
    float dacc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < N / 2; ++k) {
        regla::f2v acc = regla::f2v{dacc[(2 * k) & 3], dacc[(2 * k + 1) & 3]};
        acc = __builtin_elementwise_fma(z.p[k], z.p[k], acc);
        dacc[(2 * k) & 3] = acc.x;
        dacc[(2 * k + 1) & 3] = acc.y;
    }
    if constexpr (N & 1) dacc[(N - 1) & 3] = fmaf(ZV(z, N - 1), ZV(z, N - 1), dacc[(N - 1) & 3]);
    return (dacc[0] + dacc[1]) + (dacc[2] + dacc[3]);
}

// CRBA: one row I from its IS_I (registers)
template <int I>
HE_DEV void crba_row(regla::RegMat& M, const float (&Sj)[6], const float (&Sj2)[6], float dadd, float dadd2,
                     const float* IS) {
    using namespace regla;
    float h = lanes<smpl::kAncLo[I]>() ? dot6(Sj, IS) : 0.f;
    if constexpr (I < 64) h = lanes<1ull << I>() ? h + dadd : h;  // armature + implicit drive
    asm volatile("" : "+v"(h));
    mc_set<I>(M, h);
    if constexpr (I >= 64) {
        float h2 = lanes<(uint64_t)smpl::kAncHi[I]>() ? dot6(Sj2, IS) : 0.f;
        h2 = lanes<1ull << (I - 64)>() ? h2 + dadd2 : h2;
        asm volatile("" : "+v"(h2));
        mc2_set<I - 64>(M, h2);
    }
}

// CRBA on the matrix cores: H = IS^T S as v_mfma_f32_32x32x2_f32 tiles (rows i, columns j, K = the
// six spatial components in three steps), lower block triangle only: 6 tiles, 18 MFMAs. Operands
// come straight from LDS (lane l: IS_{32R + l%32}[2s + l/32] and S_{32C + l%32}[2s + l/32]). One
// v_permlane32_swap per register pair of a row block's column-tile pair lands "lane j holds column
// j" (RegMat), then the ancestor masks and the diagonal addends as in crba_row.
template <int RB>
HE_DEV void crba_tile_rows(regla::RegMat& M, const f32x16& ta, const f32x16& tb) {
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        const int r = RB + (v & 3) + 8 * (v >> 2);
        float a = ta[v], b = tb[v];
        swap32(a, b);  // a: row r of columns (lane), b: row r + 4
        if (r < NG) M.cp[r >> 1][r & 1] = a;
        if (r + 4 < NG) M.cp[(r + 4 < NG ? r + 4 : 0) >> 1][(r + 4) & 1] = b;
    }
}
// Entries off the ancestor chains are left as the dense product. The elimination
// reads only chain entries (an update of row I on lane j uses row K on lane j, and j in chain(I),
// I in chain(K) gives j in chain(K)), stores only chain lanes, and the pivots are diagonal, so
// those entries never reach L, D or the right-hand side; only the diagonal addends remain.
template <int I>
HE_DEV void crba_mask_rows(regla::RegMat& M, float dadd, float dadd2) {
    using namespace regla;
    if constexpr (I < NG) {
        float h = mc<I>(M);
        if constexpr (I < 64) h = lanes<1ull << I>() ? h + dadd : h;  // armature + implicit drive
        asm volatile("" : "+v"(h));
        mc_set<I>(M, h);
        if constexpr (I >= 64) {
            float h2 = mc2<I - 64>(M);
            h2 = lanes<1ull << (I - 64)>() ? h2 + dadd2 : h2;
            asm volatile("" : "+v"(h2));
            mc2_set<I - 64>(M, h2);
        }
        crba_mask_rows<I + 1>(M, dadd, dadd2);
    }
}
HE_DEV void crba_mfma(regla::RegMat& M, const Lds& L, int lane, float dadd, float dadd2) {
    const int l31 = lane & 31, kh = lane >> 5;
    float bS[3][3], aI[3][3];  // [block][k step]
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int j = 32 * c + l31;
#pragma unroll
        for (int st = 0; st < 3; ++st) {
            bS[c][st] = j < NG ? L.S[j < NG ? j : 0][2 * st + kh] : 0.f;
            aI[c][st] = j < NG ? L.IS[j < NG ? j : 0][2 * st + kh] : 0.f;
        }
    }
    const f32x16 zero = {};
    {
        f32x16 t0 = {};
#pragma unroll
        for (int st = 0; st < 3; ++st) t0 = __builtin_amdgcn_mfma_f32_32x32x2f32(aI[0][st], bS[0][st], t0, 0, 0, 0);
        crba_tile_rows<0>(M, t0, zero);  // rows 0-31 are above the diagonal for columns 32-63
    }
    {
        f32x16 t0 = {}, t1 = {};
#pragma unroll
        for (int st = 0; st < 3; ++st) {
            t0 = __builtin_amdgcn_mfma_f32_32x32x2f32(aI[1][st], bS[0][st], t0, 0, 0, 0);
            t1 = __builtin_amdgcn_mfma_f32_32x32x2f32(aI[1][st], bS[1][st], t1, 0, 0, 0);
        }
        crba_tile_rows<32>(M, t0, t1);
    }
    {
        f32x16 t0 = {}, t1 = {}, t2 = {};
#pragma unroll
        for (int st = 0; st < 3; ++st) {
            t0 = __builtin_amdgcn_mfma_f32_32x32x2f32(aI[2][st], bS[0][st], t0, 0, 0, 0);
            t1 = __builtin_amdgcn_mfma_f32_32x32x2f32(aI[2][st], bS[1][st], t1, 0, 0, 0);
            t2 = __builtin_amdgcn_mfma_f32_32x32x2f32(aI[2][st], bS[2][st], t2, 0, 0, 0);
        }
        crba_tile_rows<64>(M, t0, t1);
        // columns 64-74 (second register set, lanes 0-10): rows r from the low half, r + 4 from
        // the high half of the same tile
#pragma unroll
        for (int v = 0; v < 16; ++v) {
            const int r = 64 + (v & 3) + 8 * (v >> 2);
            float a = t2[v], b = t2[v];
            swap32(a, b);
            if (r < NG) M.cp2[(r - 64) >> 1][(r - 64) & 1] = a;
            if (r + 4 < NG) M.cp2[(r + 4 < NG ? r - 60 : 0) >> 1][(r - 60) & 1] = b;
        }
    }
    crba_mask_rows<0>(M, dadd, dadd2);
}

// one level with every parent at once: lane (group g = lane / NC, component x) takes its parent and
// children from compile-time selects, reads them (a missing child reads the parent and adds 0:
// the sum order of subtree_parent, bit-identical) and writes back; no exec-mask branch per parent
template <int J, int JE>
HE_DEV int pick_body(int g, int j0, int k) {  // k = -1: the parent, else child slot k (-1 = none)
    if constexpr (J < JE) {
        constexpr int p = smpl::kParentLevelBodies[J];
        const int v = k < 0 ? p : (k == 0 ? smpl::kChildren[p][0] : (k == 1 ? smpl::kChildren[p][1] : smpl::kChildren[p][2]));
        return g == J - j0 ? v : pick_body<J + 1, JE>(g, j0, k);
    } else {
        return -1;
    }
}
template <int NC, int D>
HE_DEV void subtree_level_flat(float* F, float* I, int lane) {
    constexpr int j0 = smpl::kParentLevelStart[D], j1 = smpl::kParentLevelStart[D + 1];
    static_assert((j1 - j0) * NC <= W, "one level's parents fit one wave");
    const int g = lane / NC, x = lane - g * NC;
    const int p = pick_body<j0, j1>(g, j0, -1);
    const int c0 = pick_body<j0, j1>(g, j0, 0), c1 = pick_body<j0, j1>(g, j0, 1), c2 = pick_body<j0, j1>(g, j0, 2);
    if (lane < (j1 - j0) * NC) {
        float* X = x < 6 ? F : I;
        const int st = x < 6 ? 6 : 10, xx = x < 6 ? x : x - 6;
        float v = X[p * st + xx];
        const float v0 = X[(c0 >= 0 ? c0 : p) * st + xx];
        const float v1 = X[(c1 >= 0 ? c1 : p) * st + xx];
        const float v2 = X[(c2 >= 0 ? c2 : p) * st + xx];
        v += c0 >= 0 ? v0 : 0.f;
        v += c1 >= 0 ? v1 : 0.f;
        v += c2 >= 0 ? v2 : 0.f;
        X[p * st + xx] = v;
    }
}
template <int NC, int D>
HE_DEV void subtree_levels(float* F, float* I, int lane) {
    if constexpr (D >= 0) {
        constexpr int j0 = smpl::kParentLevelStart[D], j1 = smpl::kParentLevelStart[D + 1];
        if constexpr (j1 > j0) {
            subtree_level_flat<NC, D>(F, I, lane);
            sync();
        }
        subtree_levels<NC, D - 1>(F, I, lane);
    }
}

// ---------------------------------------------------------------------------------- kinematics
// 2^k-th ancestor of every body (-1: none), for pointer jumping over the body tree
struct JumpTable {
    int j[4][NB];
    constexpr JumpTable() : j() {
        for (int b = 0; b < NB; ++b)
            j[0][b] = smpl::kParentBody[b] == 0 ? -1 : smpl::kParentBody[b];  // stops below the root
        for (int k = 1; k < 4; ++k)
            for (int b = 0; b < NB; ++b) j[k][b] = j[k - 1][b] < 0 ? -1 : j[k - 1][j[k - 1][b]];
    }
};
constexpr JumpTable kJumpT{};
static_assert(smpl::kNumBodyLevels <= 16, "four pointer-jumping rounds cover chains of 16 bodies");
static_assert(smpl::kNumBodyLevels - 1 <= 8, "three rounds cover the root's subtrees of depth 8");
constexpr int kKinRounds = 3;

struct Jump4 {  // the four jump targets of each body packed as bytes (LDS table BodyTopo::jump4)
    uint32_t v[NB];
    constexpr Jump4() : v() {
        for (int b = 0; b < NB; ++b)
            for (int k = 0; k < 4; ++k) v[b] |= (uint32_t)(kJumpT.j[k][b] & 0xFF) << (8 * k);
    }
};
constexpr Jump4 kJump4{};
template <int K>
HE_DEV int jump_of(uint32_t jp) {  // byte K of the lane's packed entry, sign-extended (v_bfe_i32)
    return (int)(int8_t)(jp >> (8 * K));
}

// World poses and spatial velocities, lane = body, by pointer jumping: X_b <- X_{J_k(b)} o X_b and
// V_b <- V_b + V_{J_k(b)} with J_k the 2^k-th ancestor, four rounds for chains of up to 16 bodies
// (log depth instead of a chain walk per body). X = (q, p): (qa, pa) o (qb, pb) = (qa qb, pa + Ra pb).
// The table stops below the root, so three rounds compose each chain in the root's
// frame (SMPL subtrees are 8 deep) and the root's pose / velocity / base acceleration, uniform LDS
// reads, are applied once at the end -- one dependent ds_bpermute round fewer per prefix.
// Joint axes S (lane = dof) follow from the world poses.
template <bool ACC>
HE_DEV void kinematics(Lds& L, const he_model& m, int lane, const he_sim_params& sp, bool cached) {
    const BodyTopo& T = L.T;
    const bool act = lane < NB;
    const int b = act ? lane : 0;
    const uint32_t jp = act ? T.jump4[b] : 0xFFFFFFFFu;
    f4 q;
    f3 p;
    float u[3];
    // the root's pose, read by every lane (uniform LDS addresses: broadcast)
    const f4 qr = qnormalize(f4{L.root_q[0], L.root_q[1], L.root_q[2], L.root_q[3]});
    if (b == 0) {
        q = qr;
        p = f3{0.f, 0.f, 0.f};  // origins about o
        u[0] = L.u0[0]; u[1] = L.u0[1]; u[2] = L.u0[2];
    } else {
        const int d = 3 * (b - 1);
        if (cached) {  // the previous substep's integrated rotation (pre-log)
            q = f4{L.qloc[b][0], L.qloc[b][1], L.qloc[b][2], L.qloc[b][3]};
        } else {
            q = pqexp(f3{L.q[d], L.q[d + 1], L.q[d + 2]});
            L.qloc[b][0] = q.x; L.qloc[b][1] = q.y; L.qloc[b][2] = q.z; L.qloc[b][3] = q.w;
        }
        p = f3{T.local_pos[b][0], T.local_pos[b][1], T.local_pos[b][2]};
        u[0] = L.u0[6 + d]; u[1] = L.u0[7 + d]; u[2] = L.u0[8 + d];
    }
    auto jump = [&](auto kc) {
        constexpr int K = decltype(kc)::value;
        const int j = jump_of<K>(jp);
        const int src = j < 0 ? lane : j;
        const f4 qa = f4{__shfl(q.x, src, W), __shfl(q.y, src, W), __shfl(q.z, src, W), __shfl(q.w, src, W)};
        const f3 pa = f3{__shfl(p.x, src, W), __shfl(p.y, src, W), __shfl(p.z, src, W)};
        if (j >= 0) {
            p = pa + qapply(qa, p);
            q = qmul(qa, q);
        }
    };
    jump(std::integral_constant<int, 0>{});
    jump(std::integral_constant<int, 1>{});
    jump(std::integral_constant<int, 2>{});
    if constexpr (kKinRounds == 4) jump(std::integral_constant<int, 3>{});
    if (b != 0) {  // root-frame pose of the chain -> world axes, origin about o
        p = qapply(qr, p);
        q = qmul(qr, q);
    }
    // own joint's velocity contribution: root (w0, v0 at o); joint b: (w, (p_b - o) x w), w = R_b u_b
    float V[6];
    if (b == 0) {
        V[0] = u[0]; V[1] = u[1]; V[2] = u[2]; V[3] = L.u0[3]; V[4] = L.u0[4]; V[5] = L.u0[5];
    } else {
        const f3 w = qapply(q, f3{u[0], u[1], u[2]});
        const f3 l = cross3(p, w);
        V[0] = w.x; V[1] = w.y; V[2] = w.z; V[3] = l.x; V[4] = l.y; V[5] = l.z;
    }
    float vj[6];  // the joint's own velocity S_b u_b (RNEA velocity-product term below)
#pragma unroll
    for (int x = 0; x < 6; ++x) vj[x] = V[x];
    auto vjump = [&](auto kc) {
        constexpr int K = decltype(kc)::value;
        const int j = jump_of<K>(jp);
        const int src = j < 0 ? lane : j;
        float Va[6];
#pragma unroll
        for (int x = 0; x < 6; ++x) Va[x] = __shfl(V[x], src, W);
        if (j >= 0)
#pragma unroll
            for (int x = 0; x < 6; ++x) V[x] += Va[x];
    };
    vjump(std::integral_constant<int, 0>{});
    vjump(std::integral_constant<int, 1>{});
    vjump(std::integral_constant<int, 2>{});
    if constexpr (kKinRounds == 4) vjump(std::integral_constant<int, 3>{});
    if (b != 0) {  // plus the root's own velocity
#pragma unroll
        for (int x = 0; x < 6; ++x) V[x] += L.u0[x];
    }
    if (act) {
        L.qw[b][0] = q.x; L.qw[b][1] = q.y; L.qw[b][2] = q.z; L.qw[b][3] = q.w;
        L.pw[b][0] = p.x; L.pw[b][1] = p.y; L.pw[b][2] = p.z;
        for (int x = 0; x < 6; ++x) L.V[b][x] = V[x];
    }
    if constexpr (ACC) {
        // RNEA bias acceleration (gravity as base acceleration): a_b = a_0 + sum over the chain's
        // joints j of V_j x (S_j u_j), the same prefix over the tree by pointer jumping. The base:
        // (0, v0 x w0 - g) for the free root (u = [w0, v0 at o]).
        float A[6];
        const f3 vxw = cross3(f3{L.u0[3], L.u0[4], L.u0[5]}, f3{L.u0[0], L.u0[1], L.u0[2]});
        const float A0[6] = {0.f, 0.f, 0.f, vxw.x - sp.gravity[0], vxw.y - sp.gravity[1], vxw.z - sp.gravity[2]};
        if (b == 0) {
#pragma unroll
            for (int x = 0; x < 6; ++x) A[x] = A0[x];
        } else {
            crm(V, vj, A);
        }
        auto ajump = [&](auto kc) {
            constexpr int K = decltype(kc)::value;
            const int j = jump_of<K>(jp);
            const int src = j < 0 ? lane : j;
            float Aa[6];
#pragma unroll
            for (int x = 0; x < 6; ++x) Aa[x] = __shfl(A[x], src, W);
            if (j >= 0)
#pragma unroll
                for (int x = 0; x < 6; ++x) A[x] += Aa[x];
        };
        ajump(std::integral_constant<int, 0>{});
        ajump(std::integral_constant<int, 1>{});
        ajump(std::integral_constant<int, 2>{});
        if constexpr (kKinRounds == 4) ajump(std::integral_constant<int, 3>{});
        if (b != 0) {  // plus the base acceleration
#pragma unroll
            for (int x = 0; x < 6; ++x) A[x] += A0[x];
        }
        if (act)
            for (int x = 0; x < 6; ++x) L.Acc[b][x] = A[x];
    }
    sync();
    // lane = dof: dofs 0..63 with the root's six unit axes selected in, then dofs 64..74 (ball
    // joints only); no loop and no root branch
    auto axis = [&](int i, bool may_root) {
        const bool rd = may_root && i < 6;
        const int k = rd ? 0 : i - 6;
        const int kb = k / 3, c = k - 3 * kb, bb = kb + 1;
        const f4 qb = f4{L.qw[bb][0], L.qw[bb][1], L.qw[bb][2], L.qw[bb][3]};
        const f3 e = f3{c == 0 ? 1.f : 0.f, c == 1 ? 1.f : 0.f, c == 2 ? 1.f : 0.f};
        const f3 ax = qapply(qb, e);
        const f3 l = cross3(f3{L.pw[bb][0], L.pw[bb][1], L.pw[bb][2]}, ax);
        const float g[6] = {ax.x, ax.y, ax.z, l.x, l.y, l.z};
        float* S = L.S[i];
#pragma unroll
        for (int x = 0; x < 6; ++x) S[x] = rd ? (x == i ? 1.f : 0.f) : g[x];
    };
    axis(lane, true);
    static_assert(NG - W <= W && NG - W > 0, "a second set of lanes covers dofs 64..NG-1");
    if (lane < NG - W) axis(W + lane, false);
    sync();
}

// y <- L^-1 y for the lane's rows (see regla::solve_L_rows / solve_L_gather)
HE_DEV void solve_L(const float (&r1)[regla::kRowRegs], const float (&r2)[regla::kRowRegs], int lane, float& yl,
                    float& y2) {
    (void)lane;
    regla::solve_L_rows<0>(r1, r2, yl, y2);
}

// lane i's packed row of L (dof i) and the row of dof 64 + i (lanes >= NH read row 64 and never
// use it: an exec-masked second load measured slower than the unmasked one, A/B r01)
HE_DEV void load_rows(const Lds& L, const BodyTopo& T, int lane, float (&r1)[regla::kRowRegs],
                      float (&r2)[regla::kRowRegs]) {
    const float4* p1 = reinterpret_cast<const float4*>(L.Lp + T.pack_start[lane]);
    const float4* p2 = reinterpret_cast<const float4*>(L.Lp + T.pack_start[lane < regla::NH ? 64 + lane : 0]);
#pragma unroll
    for (int q = 0; q < regla::kRowRegs / 4; ++q) {
        const float4 a1 = p1[q], a2 = p2[q];
        r1[4 * q] = a1.x; r1[4 * q + 1] = a1.y; r1[4 * q + 2] = a1.z; r1[4 * q + 3] = a1.w;
        r2[4 * q] = a2.x; r2[4 * q + 1] = a2.y; r2[4 * q + 2] = a2.z; r2[4 * q + 3] = a2.w;
    }
}

// ---------------------------------------------------------------------------------- midpoint bias
// he_sim_params.bias_midpoint (oracle/he_oracle_physics.c: substep, bias_at): the velocity-dependent
// bias (Coriolis, gyroscopic; gravity cancels) again at the midpoint velocity um = (u0 + uf) / 2 of
// the explicit step, and the free velocity corrected through the same factor:
// yh += D^-1/2 L^-T dt (bias(u0) - bias(um)). Runs between the factorisation and the contact phase,
// with the factor in Lp and the first bias's subtree forces in F. Scratch: uf (holds um), V (the
// final kinematics rewrites it), Acc (the contact phase's scratch after), Ib (own inertias, stored
// by the force pass).
// yh += D^-1/2 L^-T dc (lane = dof, then dofs 64..74 on lanes 0..10): the midpoint correction's
// forward substitution replayed from the stored factor
HE_DEV void mid_lt(Lds& L, const BodyTopo& T, int lane, float c1, float c2) {
    using regla::NH;
    __builtin_amdgcn_s_setprio(kPrioSerial);  // a serial chain: -1.2 % physics launch by A/B (r04)
    regla::solve_LT_vec_pipelined(L.Lp, T.dof_depth[lane], lane < NH ? T.dof_depth[64 + lane] : 0, c1, c2);
    __builtin_amdgcn_s_setprio(kPrioDefault);
    L.yh[lane] += c1 * L.sDinv[lane];
    if (lane < NH) L.yh[64 + lane] += c2 * L.sDinv[64 + lane];
    sync();
}

HE_DEV void bias_midpoint(Lds& L, const BodyTopo& T, int lane, const he_sim_params& p, unsigned long long* stamps,
                               unsigned long long& t_prev) {
    (void)stamps; (void)t_prev;
    using namespace regla;
    const float dt = p.dt;
    {  // um = u0 + (L^-1 D^-1/2 yh) / 2, the midpoint of u0 and the explicit free velocity
        float r1[regla::kRowRegs], r2[regla::kRowRegs];
        load_rows(L, T, lane, r1, r2);
        float t1 = L.yh[lane] * L.sDinv[lane];
        float t2 = lane < NH ? L.yh[64 + lane] * L.sDinv[64 + lane] : 0.f;
        __builtin_amdgcn_s_setprio(kPrioSerial);  // a serial chain (level sweep)
        solve_L(r1, r2, lane, t1, t2);
        __builtin_amdgcn_s_setprio(kPrioDefault);
        L.uf[lane] = L.u0[lane] + 0.5f * t1;
        if (lane < NH) L.uf[64 + lane] = L.u0[64 + lane] + 0.5f * t2;
    }
    sync();
    STAMP(25);
    const bool bl = lane < NB;
    const int b = bl ? lane : 0;
    // velocities and bias accelerations at um by pointer jumping over the chain, as the kinematics
    // does at u0 (the jump table stops below the root; the root's velocity and base acceleration are
    // added once at the end): no LDS chain walks
    float Fb[6];
    {
        const uint32_t jp = bl ? T.jump4[b] : 0xFFFFFFFFu;
        float vj[6];  // the joint's own velocity S_b um_b (the root's S are the unit axes)
        if (b == 0) {
            for (int x = 0; x < 6; ++x) vj[x] = L.uf[x];
        } else {
            const int d0 = T.dof0[b];
            const float u0_ = L.uf[d0], u1_ = L.uf[d0 + 1], u2_ = L.uf[d0 + 2];
            for (int x = 0; x < 6; ++x) vj[x] = L.S[d0][x] * u0_ + L.S[d0 + 1][x] * u1_ + L.S[d0 + 2][x] * u2_;
        }
        float V[6];
        for (int x = 0; x < 6; ++x) V[x] = vj[x];
        auto prefix6 = [&](float (&y)[6]) {
            auto round = [&](auto kc) {
                constexpr int K = decltype(kc)::value;
                const int j = jump_of<K>(jp);
                const int src = j < 0 ? lane : j;
                float ya[6];
#pragma unroll
                for (int x = 0; x < 6; ++x) ya[x] = __shfl(y[x], src, W);
                if (j >= 0)
#pragma unroll
                    for (int x = 0; x < 6; ++x) y[x] += ya[x];
            };
            round(std::integral_constant<int, 0>{});
            round(std::integral_constant<int, 1>{});
            round(std::integral_constant<int, 2>{});
            if constexpr (kKinRounds == 4) round(std::integral_constant<int, 3>{});
        };
        prefix6(V);
        const float um6[6] = {L.uf[0], L.uf[1], L.uf[2], L.uf[3], L.uf[4], L.uf[5]};
        if (b != 0)
            for (int x = 0; x < 6; ++x) V[x] += um6[x];
        const f3 vxw = cross3(f3{um6[3], um6[4], um6[5]}, f3{um6[0], um6[1], um6[2]});
        const float A0[6] = {0.f, 0.f, 0.f, vxw.x - p.gravity[0], vxw.y - p.gravity[1], vxw.z - p.gravity[2]};
        float A[6];
        if (b == 0) {
            for (int x = 0; x < 6; ++x) A[x] = A0[x];
        } else {
            crm(V, vj, A);  // joint b's velocity-product term V_b x S_b um_b
        }
        prefix6(A);
        if (b != 0)
            for (int x = 0; x < 6; ++x) A[x] += A0[x];
        float IA[6], IV[6], X[6];
        si_apply(L.Ib[b], A, IA);
        si_apply(L.Ib[b], V, IV);
        crf(V, IV, X);
        for (int x = 0; x < 6; ++x) Fb[x] = IA[x] + X[x];
    }
    sync();
    if (bl)
        for (int x = 0; x < 6; ++x) L.Acc[b][x] = Fb[x];
    sync();
    STAMP(26);
    // subtree sums of the new body forces, in place by body levels (as the first bias's): +4.8 %
    // against the per-dof-lane sums below (r03 A/B, profiles/r03/ab_pred_levels.txt, under the
    // two-wave bound that lets it fit)
    subtree_levels<6, smpl::kNumBodyLevels - 2>(&L.Acc[0][0], nullptr, lane);
    auto corr = [&](int i) {
        const int bi = i < 6 ? 0 : (i - 6) / 3 + 1;
        return dt * (dot6(L.S[i], L.F[bi]) - dot6(L.S[i], L.Acc[bi]));
    };
    float c1 = corr(lane);
    float c2 = lane < NH ? corr(64 + lane) : 0.f;
    STAMP(27);
    mid_lt(L, T, lane, c1, c2);
    STAMP(28);
}

// lane predicates of the TGS iterations' helpers as constant exec masks, rematerialised at each use
// (regla::lanes: two s_mov): a v_cmp result would be hoisted out of the iterations into an SGPR pair
// held through them, and the kernel runs out of SGPRs
HE_DEV bool lanes_body() { return regla::lanes<(1ull << NB) - 1ull>(); }        // lane < NB
HE_DEV bool lanes_hi() { return regla::lanes<(1ull << regla::NH) - 1ull>(); }   // lane < NH (dofs 64..74)
HE_DEV bool lanes_joint_dof() { return regla::lanes<~0x3Full>(); }             // lane >= 6
// ---------------------------------------------------------------------------------- TGS iterations
// he_sim_params.solver_type 1 (oracle/he_oracle_physics.c substep_tgs): the velocity-dependent bias of
// the next position iteration at the working velocity `vel` (L.u0), with the step's kinematics (S, V
// frames, own inertias Ib) -- bias_midpoint's second RNEA: the bodies' velocities and bias
// accelerations by pointer jumping, their forces, the subtree sums by body levels (L.Acc scratch: the
// contact phase's bounding spheres and patch radii are dead after the row set-up). Returns b_i = S_i . F
// for dof lane and dof 64 + lane (lanes < NH).
HE_DEV void tgs_bias_at(Lds& L, const BodyTopo& T, int lane, const he_sim_params& p, const float* vel, float& c1,
                        float& c2) {
    // in short phases through LDS (the body velocities V and joint velocities vj in the V / F words, dead
    // from the row set-up to the next kinematics), so that each phase's temporaries fit beside the
    // iterations' long-lived rows and columns
    const bool bl = lanes_body();
    const int b = bl ? lane : 0;
    const uint32_t jp = bl ? T.jump4[b] : 0xFFFFFFFFu;
    auto prefix6 = [&](float (&y)[6]) {
        auto round = [&](auto kc) {
            constexpr int K = decltype(kc)::value;
            const int j = jump_of<K>(jp);
            const int src = j < 0 ? lane : j;
            float ya[6];
#pragma unroll
            for (int x = 0; x < 6; ++x) ya[x] = __shfl(y[x], src, W);
            if (j >= 0)
#pragma unroll
                for (int x = 0; x < 6; ++x) y[x] += ya[x];
        };
        round(std::integral_constant<int, 0>{});
        round(std::integral_constant<int, 1>{});
        round(std::integral_constant<int, 2>{});
        if constexpr (kKinRounds == 4) round(std::integral_constant<int, 3>{});
    };
    {  // joint velocities vj = S_b u_b and body velocities V = prefix of vj (+ the root's)
        float vj[6];
        if (b == 0) {
            for (int x = 0; x < 6; ++x) vj[x] = vel[x];
        } else {
            const int d0 = T.dof0[b];
            const float u0_ = vel[d0], u1_ = vel[d0 + 1], u2_ = vel[d0 + 2];
            for (int x = 0; x < 6; ++x) vj[x] = L.S[d0][x] * u0_ + L.S[d0 + 1][x] * u1_ + L.S[d0 + 2][x] * u2_;
        }
        if (bl)
            for (int x = 0; x < 6; ++x) L.F[b][x] = vj[x];
        float V[6];
        for (int x = 0; x < 6; ++x) V[x] = vj[x];
        prefix6(V);
        if (b != 0)
            for (int x = 0; x < 6; ++x) V[x] += vel[x];
        if (bl)
            for (int x = 0; x < 6; ++x) L.V[b][x] = V[x];
    }
    sync();
    __builtin_amdgcn_sched_barrier(0);
    {  // bias accelerations A = prefix of V x vj (+ the base's), then the body forces
        float A[6];
        {
            const f3 vxw = cross3(f3{vel[3], vel[4], vel[5]}, f3{vel[0], vel[1], vel[2]});
            if (b == 0) {
                A[0] = 0.f; A[1] = 0.f; A[2] = 0.f;
                A[3] = vxw.x - p.gravity[0]; A[4] = vxw.y - p.gravity[1]; A[5] = vxw.z - p.gravity[2];
            } else {
                crm(L.V[b], L.F[b], A);  // joint b's velocity-product term V_b x S_b u_b
            }
        }
        prefix6(A);
        if (b != 0) {
            const f3 vxw = cross3(f3{vel[3], vel[4], vel[5]}, f3{vel[0], vel[1], vel[2]});
            A[3] += vxw.x - p.gravity[0]; A[4] += vxw.y - p.gravity[1]; A[5] += vxw.z - p.gravity[2];
        }
        float IA[6], IV[6], X[6], Vb[6];
        for (int x = 0; x < 6; ++x) Vb[x] = L.V[b][x];
        si_apply(L.Ib[b], A, IA);
        si_apply(L.Ib[b], Vb, IV);
        crf(Vb, IV, X);
        sync();
        if (bl)
            for (int x = 0; x < 6; ++x) L.Acc[b][x] = IA[x] + X[x];
    }
    sync();
    __builtin_amdgcn_sched_barrier(0);
    subtree_levels<6, smpl::kNumBodyLevels - 2>(&L.Acc[0][0], nullptr, lane);
    c1 = dot6(L.S[lane], L.Acc[dof_body(lane)]);
    c2 = lanes_hi() ? dot6(L.S[64 + lane], L.Acc[(64 + lane - 6) / 3 + 1]) : 0.f;
}

// the next position iteration's free motion: yh = D^-1/2 L^-T hs (kp (tgt - q) - c u - b) per dof (lane,
// then 64 + lane), forward substituted from the stored factor (kp parked in L.dforce during the step,
// c = hs kp + kd in L.coef, u the working velocity L.u0, b from tgs_bias_at)
HE_DEV void tgs_rhs(Lds& L, const BodyTopo& T, int lane, float hs, float c1, float c2) {
    using regla::NH;
    auto rhs = [&](int i, float b) {
        const bool jd = i >= 6;
        const int d = jd ? i - 6 : 0;
        const float drive = jd ? L.dforce[d] * (L.tgt[d] - L.q[d]) - L.coef[i] * L.u0[i] : 0.f;
        return hs * (drive - b);
    };
    float y1 = rhs(lane, c1);
    float y2 = lanes_hi() ? rhs(64 + lane, c2) : 0.f;
    __builtin_amdgcn_s_setprio(kPrioSerial);
    regla::solve_LT_vec_pipelined(L.Lp, T.dof_depth[lane], lanes_hi() ? T.dof_depth[64 + lane] : 0, y1, y2);
    __builtin_amdgcn_s_setprio(kPrioDefault);
    L.yh[lane] = y1 * L.sDinv[lane];
    if (lanes_hi()) L.yh[64 + lane] = y2 * L.sDinv[64 + lane];
    sync();
}

// the working velocity's update by one iteration: u += L^-1 D^-1/2 (yh + extra), extra = Zh^T (the
// iteration's impulse change) reduced into lane = dof (0 without contact rows)
HE_DEV void tgs_velocity(Lds& L, const BodyTopo& T, int lane, float e1, float e2) {
    using regla::NH;
    float yl = (e1 + L.yh[lane]) * L.sDinv[lane];
    float y2 = lanes_hi() ? (e2 + L.yh[64 + lane]) * L.sDinv[64 + lane] : 0.f;
    __builtin_amdgcn_s_setprio(kPrioSerial);
    regla::solve_L_streamed(L.Lp + T.pack_start[lane], L.Lp + T.pack_start[lanes_hi() ? 64 + lane : 0], yl, y2);
    __builtin_amdgcn_s_setprio(kPrioDefault);
    L.u0[lane] += yl;
    if (lanes_hi()) L.u0[64 + lane] += y2;
    sync();
}

// the iteration's implicit drive torque kp (tgt - q) - c u at its end velocity, accumulated per dof
// (lane, then 64 + lane): the reported drive force is the iterations' mean
HE_DEV void tgs_drive_acc(const Lds& L, int lane, float& f1, float& f2) {
    auto tq = [&](int i) {
        const int d = i - 6;
        return L.dforce[d] * (L.tgt[d] - L.q[d]) - L.coef[i] * L.u0[i];
    };
    if (lanes_joint_dof()) f1 += tq(lane >= 6 ? lane : 6);
    if (lanes_hi()) f2 += tq(64 + lane);
}

// ---------------------------------------------------------------------------------- fused imitation
// he_env_step's imitation step (reward / reset / observations + the device reset of flagged envs)
// as the physics kernel's epilogue, from the post-step state in LDS: the same code as the stand-alone
// imitation kernel (he_imitation_env.h), with its float32 rounding (no contraction)
constexpr int GROUP = 32;
constexpr int HOT = HE_MOTION_HOT;
constexpr int COLD = HE_MOTION_COLD;
#pragma clang fp contract(off)
#include "he_imitation_env.h"
#pragma clang fp contract(fast)

// body b's rigid-body row (he_get_buffer RB_STATE layout) from the final kinematics: origin, world
// rotation, linear velocity of the origin, angular velocity
HE_DEV SimBody body_row(const Lds& L, int b) {
    SimBody s;
    const f3 r = f3{L.pw[b][0], L.pw[b][1], L.pw[b][2]};  // about o
    s.pos = f3{L.root_pos[0], L.root_pos[1], L.root_pos[2]} + r;
    s.rot = f4{L.qw[b][0], L.qw[b][1], L.qw[b][2], L.qw[b][3]};
    const f3 w = f3{L.V[b][0], L.V[b][1], L.V[b][2]};
    s.vel = f3{L.V[b][3], L.V[b][4], L.V[b][5]} + cross3(w, r);
    s.ang = w;
    return s;
}

// ---------------------------------------------------------------------------------- integration
// Damping, the angular-velocity clamps and the semi-implicit position update over hs in one pass per
// body (lane = body). src: the solved generalized velocity (PGS: L.uf; TGS: the working velocity
// L.u0). write_out: the damped, clamped velocity becomes the state's (PGS always; TGS the last
// position iteration only: the solver's own velocity is not clamped, oracle substep_tgs). detect: the
// next substep's limit rows from the new state.
HE_DEV void integrate_bodies(Lds& L, const BodyTopo& T, int lane, const he_sim_params& p, float hs, float damp,
                             const float* src, bool write_out, bool detect) {
    // damping, the angular-velocity clamps and the semi-implicit position update in one pass per
    // body: the root composes exp(dt w) (x) q, a ball joint log(exp(q) (x) exp(dt u)); both as
    // normalize(e1 (x) e2) with the operands selected, so the two cases share one code path
    f3 lim_th = f3{0.f, 0.f, 0.f}, lim_u = f3{0.f, 0.f, 0.f};  // the joint's new q and u
    const bool bl = lanes_body();
    const bool root = regla::lanes<1ull>();
    const int d0 = root ? 0 : 6 + 3 * ((bl ? lane : 1) - 1);
    float w[3] = {src[d0] * damp, src[d0 + 1] * damp, src[d0 + 2] * damp};
    {
        // the joint's relative rate: PhysX articulation joint maxJointVelocity
        const float n2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];  // squared: the norm only where it acts
        if (!root && n2 > p.max_joint_velocity * p.max_joint_velocity) {
            const float s = p.max_joint_velocity / sqrtf(n2);
            w[0] *= s; w[1] *= s; w[2] *= s;
        }
        // the link's WORLD angular velocity (asset max_angular_velocity, PxRigidBody): w_b = w_parent +
        // R_b u_b summed along the chain (Acc is scratch here), clamped link by link; the joint rates
        // are then re-derived, u_b = R_b^T (w'_b - w'_parent) (oracle: the same pass)
        // no link can be over when |w_root| + (joints on the longest chain) x max_j |u_j| stays under
        // the cap (triangle inequality; a 1 % margin covers the prefix's rounding): the prefix and
        // the clamp are then skipped (wave-uniform), with the result they would give
        const float un = __builtin_amdgcn_sqrtf(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);  // a skip test with a 1 % margin
        const float wroot = regla::rdlane(un, 0);
        const bool may = bl && !root && un * (float)(smpl::kNumBodyLevels - 1) > 0.99f * p.max_angular_velocity - wroot;
        if (__ballot(may) != 0ull) {
        const f4 qb = bl ? f4{L.qw[lane][0], L.qw[lane][1], L.qw[lane][2], L.qw[lane][3]} : f4{0.f, 0.f, 0.f, 1.f};
        const f3 wr = root ? f3{w[0], w[1], w[2]} : qapply(qb, f3{w[0], w[1], w[2]});
        // chain prefix by pointer jumping (the table stops below the root: its rate is added last)
        f3 wo = bl ? wr : f3{0.f, 0.f, 0.f};
        {
            const uint32_t jp = bl ? T.jump4[lane] : 0xFFFFFFFFu;
            auto round = [&](auto kc) {
                constexpr int K = decltype(kc)::value;
                const int j = jump_of<K>(jp);
                const int src = j < 0 ? lane : j;
                const f3 wa = f3{__shfl(wo.x, src, W), __shfl(wo.y, src, W), __shfl(wo.z, src, W)};
                if (j >= 0) wo = wo + wa;
            };
            round(std::integral_constant<int, 0>{});
            round(std::integral_constant<int, 1>{});
            round(std::integral_constant<int, 2>{});
            if constexpr (kKinRounds == 4) round(std::integral_constant<int, 3>{});
            const f3 w0 = f3{__shfl(wr.x, 0, W), __shfl(wr.y, 0, W), __shfl(wr.z, 0, W)};
            if (bl && !root) wo = wo + w0;
        }
        const float wmax = p.max_angular_velocity;
        const float wn2 = dot3(wo, wo);
        const bool over = bl && wn2 > wmax * wmax;
        if (__ballot(over) != 0ull) {  // rare (wave-uniform branch)
            const f3 wc = over ? wo * (wmax * __builtin_amdgcn_rsqf(wn2)) : wo;
            const int pb = bl && !root ? T.chain[lane][T.depth[lane] - 1] : 0;
            const f3 wp = f3{__shfl(wc.x, pb, W), __shfl(wc.y, pb, W), __shfl(wc.z, pb, W)};
            if (bl) {
                const f3 rel = root ? wc : wc - wp;
                const f3 ub = root ? rel : qapply(qconj(qb), rel);
                w[0] = ub.x; w[1] = ub.y; w[2] = ub.z;
            }
        }
        }
    }
    if (bl) {
        if (write_out) { L.u0[d0] = w[0]; L.u0[d0 + 1] = w[1]; L.u0[d0 + 2] = w[2]; }
        const int d = root ? 0 : 3 * (lane - 1);
        const f3 dtw = f3{hs * w[0], hs * w[1], hs * w[2]};
        const f4 ed = pqexp(dtw);  // exp(q_b) itself: the kinematics' qloc (L.q is unchanged since)
        const f4 e1 = root ? ed : f4{L.qloc[lane][0], L.qloc[lane][1], L.qloc[lane][2], L.qloc[lane][3]};
        const f4 e2 = root ? f4{L.root_q[0], L.root_q[1], L.root_q[2], L.root_q[3]} : ed;
        const f4 nq = qnormalize(qmul(e1, e2));
        if (root) {
            if (write_out) { L.u0[3] = src[3]; L.u0[4] = src[4]; L.u0[5] = src[5]; }
            for (int c = 0; c < 3; ++c) L.root_pos[c] += hs * src[3 + c];
            L.root_q[0] = nq.x; L.root_q[1] = nq.y; L.root_q[2] = nq.z; L.root_q[3] = nq.w;
        } else {
            f3 nv = pqlog(nq);
            f4 nql = nq;
            if (p.joint_limits && limit_clamp(nq, nv, w)) {  // rare: the limit rows lost
                if (write_out) { L.u0[d0] = w[0]; L.u0[d0 + 1] = w[1]; L.u0[d0 + 2] = w[2]; }
                nql = pqexp(nv);
            }
            L.q[d] = nv.x; L.q[d + 1] = nv.y; L.q[d + 2] = nv.z;
            // the next substep's kinematics starts from this rotation instead of exp(log(.))
            L.qloc[lane][0] = nql.x; L.qloc[lane][1] = nql.y; L.qloc[lane][2] = nql.z; L.qloc[lane][3] = nql.w;
            lim_th = nv;
            lim_u = f3{w[0], w[1], w[2]};
        }
    }
    if (p.joint_limits && detect) limit_detect(L, lane, lane >= 1 && lane < NB, lim_th, lim_u, p);
    sync();
}

// ---------------------------------------------------------------------------------- one substep
template <bool TGS>
HE_DEV void substep(Lds& L0, const PhysArgs& a0, const he_model* mp, int lane,
                    const float* mass_scale, float mu, int tkind, unsigned long long* stamps,
                    unsigned long long& t_prev, bool first, bool last) {
    using namespace regla;
    // the launch arguments through an opaque offset too: their fields are re-read (scalar loads
    // from the kernarg segment) where used instead of being held in SGPRs across the substep loop
    int ao = 0;
    asm volatile("" : "+s"(ao));
    const PhysArgs& a = *reinterpret_cast<const PhysArgs*>(reinterpret_cast<const char*>(&a0) + ao);
    // opaque per substep: keeps the compiler from hoisting ~1k uniform model loads out of the
    // substep loop into SGPRs (which then spill into VGPR lanes)
    // (an opaque byte offset rather than an opaque pointer: the pointer keeps its global address
    // space, so the loads stay global_load / s_load instead of flat_load)
    int mo = 0;
    asm volatile("" : "+s"(mo));
    const he_model& m = *reinterpret_cast<const he_model*>(reinterpret_cast<const char*>(mp) + mo);
    // likewise an opaque VGPR base for LDS: addresses become base + immediate offset instead of
    // hundreds of hoisted uniform address constants
    int lds_off = 0;
    asm volatile("" : "+v"(lds_off));
    Lds& L = *reinterpret_cast<Lds*>(reinterpret_cast<char*>(&L0) + lds_off);
    // and the lane id: the many per-lane predicates of the unrolled algebra are then rebuilt
    // next to their use instead of being hoisted as loop invariants
    asm volatile("" : "+v"(lane));
    const BodyTopo& T = L.T;
    const he_sim_params& p = a.p;
    const float dt = p.dt;
    // TGS (solver_type 1, oracle substep_tgs): K position iterations of hs = dt / K on this step's
    // factor and contact set; PGS: one step of hs = dt
    const int K = TGS ? (p.solver_iterations < 1 ? 1 : (p.solver_iterations > kTgsMaxIt ? kTgsMaxIt : p.solver_iterations)) : 1;
    const float hs = TGS ? dt / (float)K : dt;
    __builtin_amdgcn_s_setprio(kPrioDefault);
    kinematics<true>(L, m, lane, a.p, !first);
    __builtin_amdgcn_s_setprio(kPrioDefault);
    STAMP(0);
    // ---- body spatial inertias about o + RNEA body forces (gravity as base acceleration)
    if (lane < NB) {
        int b = lane;
        float ms = mass_scale ? mass_scale[b] : 1.f;
        float mass = m.mass[b] * ms;
        f4 q = f4{L.qw[b][0], L.qw[b][1], L.qw[b][2], L.qw[b][3]};
        f3 c0, c1, c2;
        qcols(q, c0, c1, c2);
        f3 cw = qapply(q, f3{m.com[b][0], m.com[b][1], m.com[b][2]});
        f3 s = f3{L.pw[b][0], L.pw[b][1], L.pw[b][2]} + cw;  // CoM about o
        const float* in = m.inertia[b];
        float Ib[3][3] = {{in[0], in[3], in[4]}, {in[3], in[1], in[5]}, {in[4], in[5], in[2]}};
        float R[3][3] = {{c0.x, c1.x, c2.x}, {c0.y, c1.y, c2.y}, {c0.z, c1.z, c2.z}};
        float T1[3][3];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) T1[r][c] = R[r][0] * Ib[0][c] + R[r][1] * Ib[1][c] + R[r][2] * Ib[2][c];
        float I[3][3];
        float ss = dot3(s, s);
        float sv[3] = {s.x, s.y, s.z};
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c)
                I[r][c] = (T1[r][0] * R[c][0] + T1[r][1] * R[c][1] + T1[r][2] * R[c][2]) * ms +
                          mass * ((r == c ? ss : 0.f) - sv[r] * sv[c]);
        float* o10 = L.Ic[b];  // own inertia; the subtree sums accumulate in place
        o10[0] = mass; o10[1] = mass * s.x; o10[2] = mass * s.y; o10[3] = mass * s.z;
        o10[4] = I[0][0]; o10[5] = I[1][1]; o10[6] = I[2][2]; o10[7] = I[0][1]; o10[8] = I[0][2]; o10[9] = I[1][2];
        if (p.bias_midpoint)  // the body's own inertia for the midpoint's second RNEA (Ib is free until
            for (int x = 0; x < 10; ++x) L.Ib[b][x] = o10[x];  // the contact phase's segments)
        float IA[6], IV[6], X[6];
        si_apply(o10, L.Acc[b], IA);
        si_apply(o10, L.V[b], IV);
        crf(L.V[b], IV, X);
        for (int x = 0; x < 6; ++x) L.F[b][x] = IA[x] + X[x];  // body force f_b (accumulated in place)
    }
    sync();
    STAMP(1);
    // ---- subtree sums: F_b (forces) and composite inertias, in place by body levels
    __builtin_amdgcn_s_setprio(kPrioDefault);
    subtree_levels<16, smpl::kNumBodyLevels - 2>(&L.F[0][0], &L.Ic[0][0], lane);
    __builtin_amdgcn_s_setprio(kPrioDefault);
    STAMP(2);
    // ---- bias forces, IS_i = Ic S_i, drives
    const uint32_t limmask = p.joint_limits ? (uint32_t)__builtin_amdgcn_readfirstlane((int)L.limmask) : 0u;
    // lane = dof (then dofs 64..74 on lanes 0..10), the root's six dofs selected out: no loop,
    // no root branch, saturation by selects
    auto dof_terms = [&](int i, bool may_root) {
        const int b = may_root ? dof_body(i) : (i - 6) / 3 + 1;
        const float bias = dot6(L.S[i], L.F[b]);
        si_apply(L.Ic[b], L.S[i], L.IS[i]);
        const bool jd = !may_root || i >= 6;
        const int d = jd ? i - 6 : 0;
        float kp = m.stiffness[d] * p.kp_scale, kd = m.damping[d] * p.kd_scale;
        const float err = L.tgt[d] - L.q[d];
        const float u = L.u0[i];
        float tau = kp * (err - hs * u) - kd * u;
        const float lim = m.effort[d];
        // effort limit: the implicit step's drive torque, estimated with the dof's own joint-space
        // inertia H_ii = S_i . IS_i (+ armature) as tau - c dt (tau - bias) / (H_ii + dt c), scales
        // the whole drive down to the limit (oracle/he_oracle_physics.c, the drive block)
        // A joint held at its angle limit cannot give way: its check takes the torque at rest.
        const float c = hs * kp + kd;
        const float hii = dot6(L.S[i], L.IS[i]) + m.armature[d];
        const bool blocked = p.joint_limits && jd && ((limmask >> b) & 1u);
        const float tau_i = blocked ? tau : tau - c * hs * (tau - bias) * __builtin_amdgcn_rcpf(hii + hs * c);
        const float sc = fabsf(tau_i) > lim ? lim / fabsf(tau_i) : 1.f;
        tau *= sc;
        kp *= sc;
        kd *= sc;
        if (jd) L.dforce[d] = TGS ? kp : tau;  // TGS: the scaled stiffness, for the iterations' drives
        if constexpr (TGS) L.uf[i] = bias;       // TGS: the bias at u0, until an iteration re-evaluates it
        L.rhs[i] = hs * (jd ? tau - bias : -bias);
        L.coef[i] = jd ? hs * kp + kd : 0.f;
    };
    dof_terms(lane, true);
    if (lane < NG - W) dof_terms(W + lane, false);
    sync();
    STAMP(3);
    // ---- CRBA straight into registers: lane j owns column j, H[i][j] = S_j . IS_i
    RegMat M;
    {
        float Sj[6], Sj2[6];
        for (int x = 0; x < 6; ++x) { Sj[x] = L.S[lane][x]; Sj2[x] = lane < NH ? L.S[64 + lane][x] : 0.f; }
        // per-lane diagonal addend (dof = lane, and 64 + lane on lanes < 11), loaded once
        const float dadd = lane >= 6 ? m.armature[lane >= 6 ? lane - 6 : 0] + hs * L.coef[lane] : 0.f;
        const float dadd2 = lane < NH ? m.armature[lane < NH ? 58 + lane : 0] + hs * L.coef[64 + lane] : 0.f;
        (void)Sj; (void)Sj2;
        crba_mfma(M, L, lane, dadd, dadd2);
    }
    STAMP(4);
    // ---- sparse LTDL in registers (RBDA 6.5, deepest dof first); L leaves through LDS, packed
    // with the free-velocity right-hand side y = L^-T (dt*rhs) carried through the elimination
    float yl = L.rhs[lane], y2 = lane < NH ? L.rhs[64 + lane] : 0.f;
    {
        float Dl = 1.f, D2 = 1.f;
        __builtin_amdgcn_s_setprio(kPrioSerial);
        factor_pipelined(M, Dl, D2, L.Lp, L.T.dof_depth[lane], lane < NH ? L.T.dof_depth[64 + lane] : 0, yl, y2);
        __builtin_amdgcn_s_setprio(kPrioDefault);
        L.sDinv[lane] = 1.0f / sqrtf(Dl);
        if (lane < NH) L.sDinv[64 + lane] = 1.0f / sqrtf(D2);
        // the free velocity is not formed here: the contact bias takes z.u0 + zh.yh, and one L^-1
        // sweep after the solver gives uf = u0 + L^-1 D^-1/2 (yh + Zh^T lambda)
        L.yh[lane] = yl * (1.0f / sqrtf(Dl));
        if (lane < NH) L.yh[64 + lane] = y2 * (1.0f / sqrtf(D2));
    }
    sync();
    STAMP(5);
    if (!TGS && p.bias_midpoint) bias_midpoint(L, T, lane, p, stamps, t_prev);
    // the contact phase's model reads (geometry of the lane's body, self-collision pair indices)
    // depend on nothing computed here: issued now, they land behind the free-velocity sweep
    constexpr int ROUNDS = (HE_MAX_PAIRS + W - 1) / W;
    float gv[10];
    int gt;
    float grad;
    int2 prs[ROUNDS];
    const int npairs = m.num_pairs;
    {
        // body lanes their own geom, corner lanes their box's
        const int cb = L.T.cbody[lane];
        const int b = lane < NB ? lane : (cb >= 0 ? cb : 0);
        const float* g = m.geom_params[b];
#pragma unroll
        for (int i = 0; i < 10; ++i) gv[i] = g[i];
        gt = m.geom_type[b];
        grad = m.geom_radius[b];
#pragma unroll
        for (int rd = 0; rd < ROUNDS; ++rd) {
            const int pi = rd * W + lane;
            prs[rd] = *reinterpret_cast<const int2*>(m.pairs[pi < npairs ? pi : 0]);
            if (pi >= npairs) prs[rd].x = -1;
        }
    }
    sync();
    STAMP(6);
    // ---- contact slots: joint limits, terrain (bodies in order, box corners deepest-first), self
    // pairs (oracle/he_oracle_physics.c gen_contacts). Every contact generated is counted; when
    // they exceed the capacity, the limits stay and the contacts are reduced to the deepest ones
    // (smallest gap, ties in slot order), kept in slot order. The gap of each contact candidate is
    // recorded in candidate order in the IS scratch (dead after the CRBA) for that reduction.
    const int maxc = p.max_contacts < MAXC ? p.max_contacts : MAXC;
    const float off = p.contact_offset;
    const Terrain ter = terrain_of(p, tkind);
    const bool self_col = p.self_collision;
    float* gl = &L.IS[0][0];
    constexpr int kCand = 128;  // contact candidates considered by the reduction (a lying body: ~30)
    static_assert(kCand <= NG * 6, "candidate gaps fit the IS scratch");
    // the previous solve's impulses (lane = row) before the self-pair list reuses L.lam as scratch
    const float lam_prev = L.lam[lane];
    // -- joint-angle limit slots (lane = joint b - 1): the rows limit_detect flagged, re-evaluated
    // from the same state words
    int nlim = 0, nlim_all = 0;
    if (p.joint_limits) {
        const uint32_t lm = (uint32_t)__builtin_amdgcn_readfirstlane((int)L.limmask);
        const bool act = lane < NB - 1 && ((lm >> (lane + 1)) & 1u);
        const int pre = wave_prefix(act, lane, nlim_all);
        if (act && pre < maxc) {
            const int j = lane < NB - 1 ? lane : 0;
            float lg;
            f3 ld;
            angle_row(f3{L.q[3 * j], L.q[3 * j + 1], L.q[3 * j + 2]}, f3{L.u0[6 + 3 * j], L.u0[7 + 3 * j], L.u0[8 + 3 * j]},
                      p, lg, ld);
            // the row over the joint's dofs (-q^) travels in the contact position (unused by a limit)
            store_contact(L, pre, lane + 1, -2, ld * -1.f, f3{0.f, 0.f, 1.f}, lg, row_key(lane + 1, -2, 7, 0));
        }
        nlim = nlim_all < maxc ? nlim_all : maxc;
    }
    int nc = nlim;
    int terr_all = 0, self_all = 0;
    STAMP(14);
    // -- terrain candidates, one per lane-slot: a body lane (lane < 24) takes its sphere's centre or
    // its capsule's end points, a corner lane (lane 24 + 8k + c, he_topo.h corner_body) corner c of
    // the k-th box. Geometry (every lane, of its geometry body tb_):
    //  self segment P0-P1, radius rs: sphere P0 = P1 = centre; capsule from / to; box the capsule
    //    proxy along its longest axis (radius geom_radius)
    //  terrain points, radius rt: sphere the centre; capsule from, to; box corner c around its
    //    centre Pc (world centre +- the world half-axes)
    static_assert(NB % 8 == 0 && NB + 8 * HE_MAX_BOXES <= W, "corner lanes: 8-lane groups above the body lanes");
    constexpr int kPts = 2;  // terrain points per lane
    const int cbody = L.T.cbody[lane];
    const bool corner = lane >= NB && cbody >= 0;
    const int tb_ = lane < NB ? lane : (corner ? cbody : 0);
    const int cc = lane & 7;  // a corner lane's corner index
    const f3 ow = f3{L.root_pos[0], L.root_pos[1], L.root_pos[2]};  // points are about o; the terrain is world
    const bool isS = gt == HE_GEOM_SPHERE, isC = gt == HE_GEOM_CAPSULE, isB = !isS && !isC;
    float cd[kPts];
    f3 cxs[kPts], cns[kPts];
    bool cand[kPts];
    int rank[kPts];
    int myn = 0, base = 0;
    auto terrain_candidates = [&]() {
        const f4 bq = isB ? f4{gv[6], gv[7], gv[8], gv[9]} : f4{0.f, 0.f, 0.f, 1.f};
        int ax = 0;
        float emax = gv[3];
        if (gv[4] > emax) { ax = 1; emax = gv[4]; }
        if (gv[5] > emax) { ax = 2; emax = gv[5]; }
        const float half = fmaxf(emax - grad, 0.f);
        // rotations as matrices (the box's local frame and the body's world rotation): mat-vecs
        // instead of quaternion applications
        f3 bc0, bc1, bc2, wc0, wc1, wc2;
        qcols(bq, bc0, bc1, bc2);
        qcols(f4{L.qw[tb_][0], L.qw[tb_][1], L.qw[tb_][2], L.qw[tb_][3]}, wc0, wc1, wc2);
        const f3 pwb = f3{L.pw[tb_][0], L.pw[tb_][1], L.pw[tb_][2]};
        const f3 dir = (ax == 0 ? bc0 : (ax == 1 ? bc1 : bc2)) * half;
        const f3 ctr = f3{gv[0], gv[1], gv[2]};
        const f3 l0 = isB ? ctr - dir : ctr;
        const f3 l1 = isB ? ctr + dir : (isC ? f3{gv[3], gv[4], gv[5]} : ctr);
        const float rs = isS ? gv[3] : (isC ? gv[6] : grad);
        const float rt = isS ? gv[3] : (isC ? gv[6] : 0.f);
        auto rot = [&](f3 v) { return (wc0 * v.x + wc1 * v.y) + wc2 * v.z; };
        const f3 P0 = pwb + rot(l0), P1 = pwb + rot(l1);
        STAMP(18);
        if (self_col && lane < NB) {
            // world segments (the Ib scratch is dead after the subtree sums), and the bounding
            // sphere about the segment midpoint for the pair cull as one 16-byte record
            float* sg = TGS ? L.Ic[lane] : L.Ib[lane];  // TGS: Ib (own inertias) serves the iterations' bias
            sg[0] = P0.x; sg[1] = P0.y; sg[2] = P0.z; sg[3] = P1.x; sg[4] = P1.y; sg[5] = P1.z; sg[6] = rs;
            const f3 mid = (P0 + P1) * 0.5f;
            bsph(L)[lane] = make_float4(mid.x, mid.y, mid.z, 0.5f * norm3(P1 - P0) + rs);
        }
        // a corner lane's point: ((Pc +- ex) +- ey) +- ez, signs by the bits of c
        f3 X0 = P0;
        if (corner) {
            const f3 Pc = pwb + rot(ctr);
            const f3 ex = rot(bc0 * gv[3]), ey = rot(bc1 * gv[4]), ez = rot(bc2 * gv[5]);
            X0 = ((Pc + ((cc & 1) ? ex : ex * -1.f)) + ((cc & 2) ? ey : ey * -1.f)) + ((cc & 4) ? ez : ez * -1.f);
        }
        const int npts = lane < NB ? (isS ? 1 : (isC ? 2 : 0)) : (corner ? 1 : 0);
#pragma unroll
        for (int ci = 0; ci < kPts; ++ci) {
            const f3 x = ci == 0 ? X0 : P1;
            cd[ci] = terrain_dist(ter, ow + x, cns[ci]) - rt;
            cxs[ci] = x - cns[ci] * rt;
            cand[ci] = ci < npts && cd[ci] < off;
        }
        // a box keeps its 4 deepest corners (ties by index): a corner lane's rank among the 8 lanes
        // of its group, keys through xor swizzles (non-candidates keyed +inf never go first)
        const float key = corner && cand[0] ? cd[0] : __builtin_inff();
        int r = 0;
        auto beat = [&](float kj, int sx) { r += (kj < key || (kj == key && (cc ^ sx) < cc)) ? 1 : 0; };
        beat(swizzle_xor<1>(key), 1);
        beat(swizzle_xor<2>(key), 2);
        beat(swizzle_xor<3>(key), 3);
        beat(swizzle_xor<4>(key), 4);
        beat(swizzle_xor<5>(key), 5);
        beat(swizzle_xor<6>(key), 6);
        beat(swizzle_xor<7>(key), 7);
        const bool kept0 = cand[0] && (!corner || r < 4), kept1 = cand[1];
        // the kept points take the body's slots in point index order (box corners by corner index),
        // so that resting contacts keep their slots from one substep to the next (the warm start then
        // maps impulses one to one); rank[] becomes that slot offset within the body
        const uint64_t kb = __ballot(corner && kept0);
        const uint64_t bxm = __ballot(lane < NB && isB);
        const int kbox = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bxm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bxm, 0u));
        const uint32_t grp = (uint32_t)(kb >> (corner ? (lane & ~7) : (NB + 8 * (kbox < HE_MAX_BOXES ? kbox : 0)))) & 0xFFu;
        myn = lane < NB ? (isB ? __popc(grp) : (kept0 ? 1 : 0) + (kept1 ? 1 : 0)) : 0;
        // exclusive prefix of myn (0..4) over the body lanes: three bit ballots, v_mbcnt per bit
        base = 0;
        int total = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint64_t bm = __ballot((myn >> k) & 1);
            base += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u)) << k;
            total += __popcll(bm) << k;
        }
        // a corner lane starts from its box body's base
        const int bbase = __builtin_amdgcn_ds_bpermute(4 * tb_, base);
        if (corner) base = bbase;
        rank[0] = kept0 ? (corner ? __popc(grp & ((1u << cc) - 1u)) : 0) : 8;
        rank[1] = kept1 ? (kept0 ? 1 : 0) : 8;
        return total;
    };
    // the contact key's sub-index: the point's index on its body (a box's corner index)
    auto sub_of = [&](int ci) { return corner ? cc : ci; };
    // candidate gaps and bodies for the reduction (IS scratch: gaps [0, kCand), bodies (-1: a self
    // pair) [kCand, 2 kCand), the rank order [2 kCand, 3 kCand))
    int* gb = reinterpret_cast<int*>(gl + kCand);
    int* gord = reinterpret_cast<int*>(gl + 2 * kCand);
    static_assert(3 * kCand <= NG * 6, "reduction scratch fits IS");
    int rows_terr = 0;  // solver rows of every terrain candidate kept (patch friction)
    {
        terr_all = terrain_candidates();
        STAMP(16);
        // candidate k = base + rank (in slot order): its gap for the reduction, its slot nlim + k
#pragma unroll
        for (int ci = 0; ci < kPts; ++ci) {
            if (cand[ci] && rank[ci] < 4) {
                const int k = base + rank[ci];
                if (k < kCand) { gl[k] = cd[ci]; gb[k] = tb_; }
                if (nlim + k < maxc)
                    store_contact(L, nlim + k, tb_, -1, cxs[ci], cns[ci], cd[ci], row_key(tb_, -1, sub_of(ci), 0));
            }
        }
        // rows of the body's patch: k points, k normal rows + 2 tangential (+ 1 torsional from k = 2)
        const int pr = myn == 0 ? 0 : myn + (myn >= 2 ? 3 : 2);
#pragma unroll
        for (int k = 0; k < 3; ++k) rows_terr += __popcll(__ballot((pr >> k) & 1)) << k;
        nc = nlim + terr_all < maxc ? nlim + terr_all : maxc;
        if (lane < NB) {  // the body's slot range, for the per-body force sums
            const int s0 = nlim + base;
            L.tbase[lane] = (int8_t)(s0 < maxc ? s0 : maxc);
            L.tcnt[lane] = (int8_t)(s0 + myn < maxc ? myn : (s0 < maxc ? maxc - s0 : 0));
        }
        if (lane == 0) L.nterr = nc;
    }
    STAMP(17);
    // -- self pairs: broad phase (bounding spheres, survivors compacted in pair order into the lam
    // scratch), narrow phase W survivors per pass; `visit(hit, i, j, x, n, gap, k)` gets every hit
    // with its candidate index k (in pair order after the terrain candidates)
    auto self_pairs = [&](auto visit) {
        sync();
        int* list = reinterpret_cast<int*>(L.lam);
        auto compact = [&](int skip) {  // survivors skip .. skip + W - 1 into the list
            int k = 0;
#pragma unroll
            for (int rd = 0; rd < ROUNDS; ++rd) {
                const int i = prs[rd].x, j = prs[rd].y;
                bool need = false;
                if (i >= 0) {
                    const float4 bi = bsph(L)[i], bj = bsph(L)[j];
                    const f3 d = f3{bi.x - bj.x, bi.y - bj.y, bi.z - bj.z};
                    const float lim = bi.w + bj.w + off + 1e-3f;
                    need = dot3(d, d) < lim * lim;
                }
                const uint64_t bm = __ballot(need);
                const int slot = k + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u)) - skip;
                if (need && slot >= 0 && slot < W) list[slot] = (rd * W + lane) | (i << 16) | (j << 24);
                k += __popcll(bm);
            }
            sync();
            return k;
        };
        // broad phase: a pair whose bounding spheres (segment midpoint, half length + radius) are
        // apart by more than the contact offset plus a 1 mm guard cannot reach gap < offset
        const int nsurv = compact(0);
        STAMP(19);
        int nhit = 0;
        for (int s0 = 0; s0 < nsurv; s0 += W) {
            bool hit = false;
            f3 px = f3{0.f, 0.f, 0.f}, pn = f3{0.f, 0.f, 0.f};
            float pgap = 0.f;
            int i = 0, j = 0;
            if (s0 + lane < nsurv) {
                const int e = list[lane];
                i = (e >> 16) & 0xFF;
                j = (e >> 24) & 0xFF;
                const float* si = TGS ? L.Ic[i] : L.Ib[i];
                const float* sj = TGS ? L.Ic[j] : L.Ib[j];
                const float ri = si[6], rj = sj[6];
                f3 ci, cj;
                seg_seg(f3{si[0], si[1], si[2]}, f3{si[3], si[4], si[5]}, f3{sj[0], sj[1], sj[2]}, f3{sj[3], sj[4], sj[5]}, ci, cj);
                const f3 dv = ci - cj;
                const float len = norm3(dv);
                pgap = len - ri - rj;
                if (pgap < off) {
                    hit = true;
                    pn = len > 1e-9f ? dv * __builtin_amdgcn_rcpf(len) : f3{0.f, 0.f, 1.f};
                    px = cj + pn * (rj + 0.5f * pgap);
                }
            }
            int total;
            const int pre = wave_prefix(hit, lane, total);
            visit(hit, i, j, px, pn, pgap, terr_all + nhit + pre);
            nhit += total;
            if (s0 + W < nsurv) compact(s0 + W);  // more than W survivors: the next pass (rare)
        }
        return nhit;
    };
    if (self_col) {
        self_all = self_pairs([&](bool hit, int i, int j, f3 px, f3 pn, float pgap, int k) {
            if (hit && k < kCand) { gl[k] = pgap; gb[k] = -1; }
            if (hit && nlim + k < maxc) store_contact(L, nlim + k, i, j, px, pn, pgap, row_key(i, j, 0, 0));
        });
        nc = nlim + terr_all + self_all < maxc ? nlim + terr_all + self_all : maxc;
    }
    const int ncand_all = nlim_all + terr_all + self_all;
    if ((nlim + terr_all + self_all > maxc || nlim + rows_terr + 3 * self_all > MAXR) && nlim < maxc) {
        // ---- overflow (rare, wave-uniform): past the slots or the solver rows. The contacts are
        // taken deepest first (smallest gap, ties in slot order), each kept while its rows still fit
        // (a self pair or a body's first terrain point 3, its second 2, 1 after: oracle gen_contacts),
        // and the kept ones are regenerated in slot order
        sync();
        const int keep = maxc - nlim;
        const int T = terr_all + self_all < kCand ? terr_all + self_all : kCand;
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // each candidate's depth rank -> the rank order
            const int k = h * W + lane;
            if (k < T) {
                const float gk = gl[k];
                int r = 0;
                for (int jj = 0; jj < T; ++jj) {  // uniform LDS reads (broadcast)
                    const float g2 = gl[jj];
                    r += (g2 < gk || (g2 == gk && jj < k)) ? 1 : 0;
                }
                gord[r] = k;
            }
        }
        sync();
        // the greedy pass in rank order (wave-uniform): candidate and body from registers by
        // v_readlane, the kept points per body in lane = body
        const int ko0 = lane < T ? gord[lane] : 0, ko1 = W + lane < T ? gord[W + lane < kCand ? W + lane : 0] : 0;
        const int kb0 = gb[ko0], kb1 = gb[ko1];
        uint64_t km[2] = {0ull, 0ull};
        int rows = nlim, kept_n = 0, pcnt = 0;
        for (int q = 0; q < T; ++q) {
            const int k = q < W ? __builtin_amdgcn_readlane(ko0, q & (W - 1)) : __builtin_amdgcn_readlane(ko1, q & (W - 1));
            const int b = q < W ? __builtin_amdgcn_readlane(kb0, q & (W - 1)) : __builtin_amdgcn_readlane(kb1, q & (W - 1));
            const int pc = b >= 0 ? __builtin_amdgcn_readlane(pcnt, b) : 0;
            const int cost = b < 0 ? 3 : (pc == 0 ? 3 : (pc == 1 ? 2 : 1));
            if (kept_n < keep && rows + cost <= MAXR) {
                rows += cost;
                ++kept_n;
                pcnt += lane == b ? 1 : 0;
                if (k < W) km[0] |= 1ull << (k & (W - 1));
                else km[1] |= 1ull << (k & (W - 1));
            }
        }
        auto before = [&](int k) {  // kept candidates below index k
            const uint64_t lo = k >= W ? km[0] : (k <= 0 ? 0ull : km[0] & ((~0ull) >> (W - k)));
            const uint64_t hi = k <= W ? 0ull : (k >= 2 * W ? km[1] : km[1] & ((~0ull) >> (2 * W - k)));
            return __popcll(lo) + __popcll(hi);
        };
        auto is_kept = [&](int k) { return k < 2 * W && ((km[k >= W ? 1 : 0] >> (k & (W - 1))) & 1ull); };
        terrain_candidates();
#pragma unroll
        for (int ci = 0; ci < kPts; ++ci) {
            if (cand[ci] && rank[ci] < 4) {
                const int k = base + rank[ci];
                if (is_kept(k))
                    store_contact(L, nlim + before(k), tb_, -1, cxs[ci], cns[ci], cd[ci], row_key(tb_, -1, sub_of(ci), 0));
            }
        }
        if (lane < NB) {
            const int s0 = nlim + before(base);
            L.tbase[lane] = (int8_t)s0;
            L.tcnt[lane] = (int8_t)(nlim + before(base + myn) - s0);
        }
        if (lane == 0) L.nterr = nlim + before(terr_all);
        if (self_col) {
            self_pairs([&](bool hit, int i, int j, f3 px, f3 pn, float pgap, int k) {
                if (hit && is_kept(k)) store_contact(L, nlim + before(k), i, j, px, pn, pgap, row_key(i, j, 0, 0));
            });
        }
        nc = nlim + before(T);
    }
    STAMP(15);
    if (lane == 0) { L.nc = nc; L.nlim = nlim; L.ncand = ncand_all; }
    if (lane < NB) { L.cf[lane][0] = 0.f; L.cf[lane][1] = 0.f; L.cf[lane][2] = 0.f; }
    sync();
    // ---- solver rows (patch friction, oracle build_rows), lane = slot: a joint limit 1 row, a point
    // its normal row, the last point of a body's terrain patch then the patch's 2 tangential rows
    // (+ 1 torsional from 2 points on), a self pair its normal and 2 tangential rows; the row table
    // (row -> slot, kind) by the slots' exclusive prefix
    int nr = 0;
    {
        const bool on = lane < nc;
        const int bb = on ? L.cbb[lane < MAXC ? lane : 0] : 0;
        const int b0 = bb & 0xFF, b1 = (bb >> 8) - 2;
        int cost = 0;
        if (on) {
            if (b1 == -2) cost = 1;
            else if (b1 >= 0) cost = 3;
            else {
                const int tn = L.tcnt[b0];
                cost = lane == L.tbase[b0] + tn - 1 ? 1 + (tn >= 2 ? 3 : 2) : 1;
            }
        }
        int start = 0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const uint64_t bm = __ballot((cost >> k) & 1);
            start += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u)) << k;
            nr += __popcll(bm) << k;
        }
        if (on) {
            L.srow0[lane < MAXC ? lane : 0] = (int8_t)start;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (k < cost) { L.rslot[start + k] = (int8_t)lane; L.rkind[start + k] = (int8_t)k; }
        }
    }
    // ---- each body's terrain patch (lane = body, tcnt > 0): normal = the normalised sum of its
    // points' normals, the points' centroid (about o) and the torsion radius (mean tangential
    // distance of the points from the centroid), into the RNEA force scratch F (dead from the
    // midpoint bias to the next substep's force pass) and the Acc words after the bounding spheres
    float* prad = &L.Acc[0][0] + 4 * NB;
    static_assert(5 * NB <= 6 * NB, "patch radii fit Acc after the bounding spheres");
    if (lane < NB && L.tcnt[lane] > 0) {
        const int p0 = L.tbase[lane], pc = L.tcnt[lane];
        f3 px[4];
        f3 np = f3{0.f, 0.f, 0.f}, xp = f3{0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int sj = j < pc ? p0 + j : p0;
            px[j] = f3{L.cx[sj][0], L.cx[sj][1], L.cx[sj][2]};
            if (j < pc) {
                np = np + f3{L.cn[sj][0], L.cn[sj][1], L.cn[sj][2]};
                xp = xp + px[j];
            }
        }
        np = np * (1.0f / norm3(np));
        xp = xp * (1.0f / (float)pc);
        float rp = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const f3 d = px[j] - xp;
            const f3 tg = d - np * dot3(d, np);
            if (j < pc) rp += norm3(tg);
        }
        float* pf = L.F[lane];
        pf[0] = np.x; pf[1] = np.y; pf[2] = np.z; pf[3] = xp.x; pf[4] = xp.y; pf[5] = xp.z;
        prad[lane] = rp * (1.0f / (float)pc);
    }
    sync();
    STAMP(7);
    // ---- each row's Jacobian data (lane = row): slot, kind, bodies; a friction row's patch (a
    // body's terrain points [tbase, tbase + tcnt), or the self pair alone): normal = the normalised
    // sum of the points' normals, the tangent basis of it, the points' centroid, the torsion radius
    // (mean tangential distance of the points from the centroid); its normal rows n0 .. n0 + cnt - 1
    // as a lane mask, its bound weight muw (mu, or mu r for the torsional row), its 16-bit key
    const bool act = lane < nr;
    const int rs_ = act ? L.rslot[lane] : 0;
    const int kind = act ? L.rkind[lane] : 0;
    const int rbb = L.cbb[rs_];
    const int rb0 = rbb & 0xFF, rb1 = (rbb >> 8) - 2;
    // the row's 16-bit key: a normal row its slot's, a friction row its patch's (terrain: the body's
    // patch, HE_KEY_PATCH) with the kind
    const int rkey = kind == 0 ? L.ckey[rs_]
                               : ((rb1 == -1 ? row_key(rb0, -1, HE_KEY_PATCH, 0) : L.ckey[rs_]) | (kind << 14));
    // ---- warm start: the previous solve's impulse of each row's key (lane r matches its key against
    // the old keys by readlane and fetches the impulse)
    float lam0 = 0.f;
    {
        const int nw = __builtin_amdgcn_readfirstlane(L.nwc);
        if (nw > 0 && nr > 0) {
            const int wk = lane < nw ? L.wckey[lane] : -1;
            const int ck = act ? rkey : -2;
            if (nw == nr && __ballot(act && wk != ck) == 0ull) {
                lam0 = act ? lam_prev : 0.f;  // the same rows in the same order (at rest)
            } else {
                int src = -1;
                for (int j = 0; j < nw; ++j) {
                    const int kj = __builtin_amdgcn_readlane(wk, j);
                    src = (src < 0 && kj == ck) ? j : src;
                }
                const float v = __shfl(lam_prev, src >= 0 ? src : 0, W);
                lam0 = (act && src >= 0) ? v : 0.f;
            }
        }
        // the old keys are matched: this solve's row keys replace them (the next solve's warm start)
        L.wckey[lane] = act ? rkey : -1;
    }
    f3 dd, rho;
    {
        const f3 xs = f3{L.cx[rs_][0], L.cx[rs_][1], L.cx[rs_][2]};
        const f3 ns = f3{L.cn[rs_][0], L.cn[rs_][1], L.cn[rs_][2]};
        // a friction row's patch: the body's terrain patch (above), or a self pair's own point
        const bool terr = rb1 == -1;
        const float* pf = L.F[rb0];
        const f3 np = terr ? f3{pf[0], pf[1], pf[2]} : ns;
        const f3 xp = terr ? f3{pf[3], pf[4], pf[5]} : xs;
        const float rp = terr ? prad[rb0] : 0.f;
        f3 t1, t2;
        friction_basis(np, t1, t2);
        dd = kind == 0 ? ns : (kind == 1 ? t1 : (kind == 2 ? t2 : f3{0.f, 0.f, 0.f}));
        rho = kind == 3 ? np : cross3(kind == 0 ? xs : xp, dd);  // contact points about o
        // the friction bound weight, parked in the impulse words (dead from the self-pair list to
        // the solve's store) until the PGS: a short live range through the rows' register peak
        L.lam[lane] = act && kind > 0 ? (kind == 3 ? mu * rp : mu) : 0.f;
        // the row's linear direction for the reported forces (IS scratch, read after the solve; a
        // joint limit's and a torsional row's: none)
        if (act) {
            float* fr = gl + 2 * kCand;
            const bool none = rb1 == -2;
            fr[3 * lane] = none ? 0.f : dd.x;
            fr[3 * lane + 1] = none ? 0.f : dd.y;
            fr[3 * lane + 2] = none ? 0.f : dd.z;
        }
    }
    static_assert(2 * kCand + 3 * W <= NG * 6, "per-row force directions fit IS");
    const float damp = 1.0f / (1.0f + dt * p.angular_damping);
    float tf1 = 0.f, tf2 = 0.f;  // TGS: the iterations' drive torques, summed per dof (lane, 64 + lane)
    // TGS: what follows a position iteration's velocity update: its drive torques, the positions by hs
    // (the last iteration: the step's output velocity), then (not the last) the next iteration's bias
    // and free motion
    auto tgs_advance = [&](int it) {
        const bool lastit = it + 1 == K;
        tgs_drive_acc(L, lane, tf1, tf2);
        integrate_bodies(L, T, lane, p, hs, damp, L.u0, lastit, lastit && !last);
        __builtin_amdgcn_sched_barrier(0);
        STAMP(12);
        if (!lastit) {
            // the velocity-dependent bias: re-evaluated at the start of every second iteration (oracle
            // g_bias_every: as stable as every iteration at half the passes), else the one in L.uf
            if (p.bias_midpoint && ((it + 1) % kTgsBiasEvery) == 0) {
                float b1, b2;
                tgs_bias_at(L, T, lane, p, L.u0, b1, b2);
                L.uf[lane] = b1;
                if (lane < NH) L.uf[64 + lane] = b2;
            }
            const float c1 = L.uf[lane];
            const float c2 = lane < NH ? L.uf[64 + lane] : 0.f;
            __builtin_amdgcn_sched_barrier(0);
            STAMP(29);
            tgs_rhs(L, T, lane, hs, c1, c2);
            __builtin_amdgcn_sched_barrier(0);
            STAMP(30);
        }
    };
    // TGS: the reported drive force, the iterations' mean (the joint-limit force is added by the caller)
    auto tgs_drive_out = [&]() {
        if (lane >= 6) L.dforce[lane >= 6 ? lane - 6 : 0] = tf1 / (float)K;
        if (lane < NH) L.dforce[58 + lane] = tf2 / (float)K;
        sync();
    };
    if (nr > 0) {
        // ---- contact rows, one per lane: z = J_r^T, brow = J_r uf + bias, then z <- D^-1/2 L^-T z
        // (dofs outside every row's support stay zero and are skipped wave-uniformly), so that the
        // Delassus operator A = Zh Zh^T is a plain Gram matrix of the lanes' registers
        float brow = 0.f, diag = 0.f, lamv = 0.f;
        float acol[MAXR];  // lane c: A[r][c]
        regla::ZVec z;     // lane r: row r of Zh = D^-1/2 L^-T J^T, kept for du = L^-1 D^-1/2 Zh^T lambda
        bool legs;         // every row's support inside the root and the legs (wave-uniform)
        {
            const uint32_t anc0 = act ? T.anc_mask[rb0] : 0u;
            const uint32_t anc1 = (act && rb1 >= 0) ? T.anc_mask[rb1] : 0u;
            // bodies on some row's support (wave-uniform): the only ones whose dofs can be nonzero
            const uint32_t lb = wave_or(anc0 | anc1);
            legs = (lb & ~kLegBodies) == 0u && !a.full_dofs;
            // z = J_r^T and brow = J_r u0 on the matrix cores
            zrows_mfma(z, lb, anc0, anc1, rho, dd, L, lane, nr <= 32);
            // joint-limit rows: the stored row over the joint's three dofs (its support is the joint's
            // ancestor chain, anc0)
            const bool limrow = act && rb1 == -2;
            if (__ballot(limrow)) {  // wave-uniform
                const int bl = limrow ? rb0 : 0;
                const float g3[3] = {L.cx[rs_][0], L.cx[rs_][1], L.cx[rs_][2]};
#pragma unroll
                for (int i = 0; i < NG; ++i) {
                    const float v = i < 6 ? 0.f : (bl == (i < 6 ? 0 : (i - 6) / 3 + 1) ? g3[i < 6 ? 0 : (i - 6) % 3] : 0.f);
                    ZV(z, i) = limrow ? v : ZV(z, i);
                }
            }
            // J_r u0 on the register pairs (dof i into sum i mod 4); over the legs' dofs only when every
            // row's support is there (the dropped terms are fma(0, u, s) = s: the same bits)
            brow = (HE_TGS_LEGS_ROWS && legs) ? zdot_lds<KZ>(z, L.u0) : zdot_lds<NG>(z, L.u0);
            if (act && kind == 0) {
                const float g = L.cgap[rs_];
                // speculative: close within the solve's step; penetrating: recover at baumgarte per physics
                // step (TGS too: oracle contact_bias)
                brow += g >= 0.f ? g / hs : fmaxf(p.baumgarte * g / dt, -p.max_depenetration_velocity);
            }
            STAMP(20);
            __builtin_amdgcn_s_setprio(kPrioSerial);
            zbs<NG - 1>(L.Lp, z, lb);
            __builtin_amdgcn_s_setprio(kPrioDefault);
            STAMP(21);
            // z <- D^-1/2 z: the scale of dof i is broadcast from lane i's register (no LDS)
            const float sdl = L.sDinv[lane], sdl2 = lane < NH ? L.sDinv[64 + lane] : 0.f;
            // then |zh_r|^2 and J_r (uf - u0) = zh_r . yh, yh_i broadcast from lane i (v_readlane: no LDS
            // loads to hoist into registers at the phase's register peak), four lanes per block into
            // four SGPRs (one hazard nop per block; through one SGPR the 75 products serialised: this
            // phase -10 %, the launch -0.5 % by A/B, bit-identical, round 4). Leg support: dofs 0..KZ-1
            // (zh is exactly zero past them: the same bits)
            const float yhl = L.yh[lane];
            if (HE_TGS_LEGS_ROWS && legs) {
                scale_rows<0, KZ>(z, sdl, sdl2);
                diag = znorm2<KZ>(z);
                brow += zdot_lanes_legs(z, yhl);
            } else {
                scale_rows<0>(z, sdl, sdl2);
                diag = znorm2<NG>(z);
                brow += zdot_lanes(z, yhl, lane < NH ? L.yh[64 + lane] : 0.f);
            }
            // dof groups of four touching a support body (wave-uniform, from lb)
            uint32_t live = 0u;
#pragma unroll
            for (int g = 0; g < NGRP; ++g)
                if (lb & kGroupBodies[g]) live |= 1u << g;
            STAMP(8);
            // ---- Delassus columns on the matrix cores: A[r][c] = sum_i zh_r[i] zh_c[i]
            if (nr <= 32) delassus_mfma32(z, acol, live);  // wave-uniform
            else if (nr <= 48) delassus_mfma48(z, acol, live);
            else delassus_mfma(z, acol, live);
        }
        STAMP(9);
        if constexpr (TGS) {
            // ---- TGS position iterations (oracle substep_tgs): each one Gauss-Seidel sweep on the
            // accumulated impulses, started from them plus the previous iteration's change (the first:
            // the cached change of the previous step), against J u of the iteration's free velocity and
            // the bias of the row's separation, advanced by hs J_r u after each iteration
            const float invd = 1.0f / (act ? diag + 1e-12f : 1.f);
            const float ninvd = -invd;
            const int nrb = __builtin_amdgcn_readfirstlane(nr);
            // the first iteration starts from the cached (previous step's) impulses' per-iteration share g0;
            // its residual w = brow + A g0 (lane c of acol holds A[r][c] = A[c][r])
            const float g0 = lam0 * (1.0f / (float)K);
            float w0 = brow;
            if (__ballot(g0 != 0.f)) {  // wave-uniform; rows >= nr hold no impulse
                auto aw = [&](auto nrows) {
                    constexpr int NRW = decltype(nrows)::value;
                    float wa[4] = {0.f, 0.f, 0.f, 0.f};
                    regla::static_for<0, NRW, 4>([&](auto rc) {
                        constexpr int r0 = decltype(rc)::value;
                        float sv[4];
                        regla::rdlane4<r0>(g0, sv);
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (r0 + q < NRW) wa[(r0 + q) & 3] = fmaf(acol[r0 + q < NRW ? r0 + q : 0], sv[q], wa[(r0 + q) & 3]);
                    });
                    w0 += (wa[0] + wa[1]) + (wa[2] + wa[3]);
                };
                if (nrb <= 16) aw(std::integral_constant<int, 16>{});
                else if (nrb <= 32) aw(std::integral_constant<int, 32>{});
                else if (nrb <= 48) aw(std::integral_constant<int, 48>{});
                else aw(std::integral_constant<int, MAXR>{});
            }
            float dl = 0.f;
            // the iterations, for one row-count class of columns held in registers (<= 32 rows: a
            // standing body's 28; more: the 63-row form), so that the common case keeps 31 registers free
            // for the phases between the sweeps
            auto tgs_solve = [&](auto ncls) {
            constexpr int NC = decltype(ncls)::value;
            // the iterations' Zh products over dofs 0..KZ-1 when every row's support is in the legs: a
            // wave-uniform branch inside the one instantiation (its own instantiation, with Zh's other 44
            // registers dead, ran the standing body as fast but every other env 1-2 % slower: the
            // second copy of the loop body; profiles/r06/ab_tgs_legs.txt)
            const bool legs_it = HE_TGS_LEGS && NC == 32 && legs;
            // the sweep's columns -A[r][lane] / A[lane][lane] of the class's rows; up to 32 rows packed
            // with their bound weights as the PGS sweep's (pgs_sweep_fix), past 32 the weights rebuilt
            // per row (pgs_sweep_tgs: 63 registers fewer)
            constexpr bool PACK = NC <= 32;
            float ap[PACK ? 1 : NC];
            regla::f2v ak[PACK ? NC : 1];
            const bool isn = kind == 0;
            const float muw = L.lam[lane];  // the friction bound weight parked by the row set-up
            uint32_t mlo = 0u, mhi = 0u;
            if (act && !isn) {
                const int pc = rb1 == -1 ? L.tcnt[rb0] : 1;
                const uint64_t pm = ((1ull << pc) - 1ull) << (lane - (kind - 1) - pc);
                mlo = (uint32_t)pm;
                mhi = (uint32_t)(pm >> 32);
            }
            const int n0 = act && !isn ? (int)__builtin_ctzll(((uint64_t)mhi << 32) | mlo) : 0;
            {
                auto prep = [&](auto r0c) {
                    constexpr int R0 = decltype(r0c)::value;
#pragma unroll
                    for (int r = R0; r < (R0 + 16 < NC ? R0 + 16 : NC); ++r) {
                        if constexpr (PACK) {
                            const int sel = __builtin_amdgcn_sbfe((int)(r < 32 ? mlo : mhi), r & 31, 1);
                            ak[r] = regla::f2v{acol[r] * ninvd, __int_as_float(sel & __float_as_int(muw))};
                        } else {
                            ap[r] = acol[r] * ninvd;
                        }
                    }
                };
                prep(std::integral_constant<int, 0>{});
                if (nrb > 16) prep(std::integral_constant<int, 16>{});
                if constexpr (NC > 32) {
                    if (nrb > 32) prep(std::integral_constant<int, 32>{});
                    if (nrb > 48) prep(std::integral_constant<int, 48>{});
                }
            }
            auto patch_bound = [&](float lv) {  // muw x the patch's normal impulses (<= 4 rows)
                float bnd = 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float v = __shfl(lv, (n0 + j) & (W - 1), W);
                    const int bit = n0 + j;
                    const bool in = bit < 32 ? ((mlo >> (bit & 31)) & 1u) : ((mhi >> (bit & 31)) & 1u);
                    bnd += in ? v : 0.f;
                }
                return bnd * muw;
            };
            auto gbias = [&](float g) {
                return g >= 0.f ? g / hs : fmaxf(p.baumgarte * g / dt, -p.max_depenetration_velocity);
            };
            const float kInf = __builtin_inff();
            float sep = act && isn ? L.cgap[rs_] : 0.f;  // the row's separation (a limit row: its angle gap)
            float bb = act && isn ? gbias(sep) : 0.f;   // its bias (brow holds it)
            float applied = 0.f;                         // the impulse already in the working velocity
            lamv = g0;
            float cd = act ? -w0 * invd : 0.f;
            float bnd = patch_bound(lamv);
            float lo = isn ? -lamv : -bnd - lamv;
            float hi = isn ? kInf : bnd - lamv;
            const int nru = __builtin_amdgcn_readfirstlane(nr);
            for (int it = 0; it < K; ++it) {
                float dvec = 0.f;
                int nrs = nru;
                asm volatile("" : "+s"(nrs));
                regla::f2v ch = {cd, hi};
                __builtin_amdgcn_s_setprio(kPrioSerial);
                if constexpr (PACK) {
                    if (nrs <= 16) pgs_sweep_fix<0, 16, NC>(ch, dvec, lo, ak, nrs);
                    else pgs_sweep_fix<0, 32, NC>(ch, dvec, lo, ak, nrs);
                } else {
                    if (nrs <= 48) pgs_sweep_tgs<0, 48, NC>(ch, dvec, lo, ap, mlo, mhi, muw, nrs);
                    else pgs_sweep_tgs<0, MAXR, NC>(ch, dvec, lo, ap, mlo, mhi, muw, nrs);
                }
                __builtin_amdgcn_s_setprio(kPrioDefault);
                STAMP(10);
                cd = ch.x;
                lamv += dvec;
                dl = act ? lamv - applied : 0.f;  // this iteration's impulse change
                applied = lamv;
                const float v = act ? -cd * (diag + 1e-12f) - bb : 0.f;  // J_r u after the sweep
                float e1, e2;  // Zh^T dl, lane = dof (and 64 + lane): also the next start's A dl = Zh (Zh^T dl)
                __builtin_amdgcn_sched_barrier(0);  // phase fences: each phase's temporaries beside the
                if (legs_it) {                          // loop's long-lived rows and columns, not several
                    e1 = reduce_scatter_z_legs(z, dl);
                    e2 = 0.f;
                } else {
                    reduce_scatter_z(z, dl, lane, e1, e2);
                }
                __builtin_amdgcn_sched_barrier(0);
                e2 = lane < NH ? e2 : 0.f;
                tgs_velocity(L, T, lane, e1, e2);  // the working velocity: u += L^-1 D^-1/2 (yh + Zh^T dl)
                __builtin_amdgcn_sched_barrier(0);
                STAMP(11);
                if (isn) sep += hs * v;
                const bool lastit = it + 1 == K;
                tgs_advance(it);
                __builtin_amdgcn_sched_barrier(0);
                if (!lastit) {
                    // the next sweep's start about lambda = applied + dl: w = J u + zh . yh + bias(sep) + A dl,
                    // with zh . yh + A dl = zh . (yh + Zh^T dl), one dot product
                    const float yhl = L.yh[lane] + e1;
                    float zy;
                    if (legs_it) {
                        zy = zdot_lanes_legs(z, yhl);
                    } else {
                        const float yh2 = lane < NH ? L.yh[64 + lane] + e2 : 0.f;
                        zy = zdot_lanes(z, yhl, yh2);
                    }
                    bb = act && isn ? gbias(sep) : 0.f;
                    lamv = applied + dl;
                    cd = act ? -(v + zy + bb) * invd : 0.f;
                    bnd = patch_bound(lamv);
                    lo = isn ? -lamv : -bnd - lamv;
                    hi = isn ? kInf : bnd - lamv;
                    STAMP(31);
                }
            }
            };
            if (nrb <= 32) tgs_solve(std::integral_constant<int, 32>{});
#ifdef HE_TGS_CLASS32_ONLY  // diagnostic A/B only (wrong past 32 rows): what the 63-row class costs the common path
            else tgs_solve(std::integral_constant<int, 32>{});
#else
            else tgs_solve(std::integral_constant<int, MAXR>{});
#endif
            // the cache and the reported forces take the step's accumulated impulses
            L.lam[lane] = act ? lamv : 0.f;
            if (lane == 0) L.nwc = p.warm_start ? nr : 0;
            tgs_drive_out();
            // the joint-limit force (dof_force = drive and limit together): limit row c = slot c
            const int nl = __builtin_amdgcn_readfirstlane(L.nlim);
            if (lane < nl) {
                const int d0 = 3 * ((L.cbb[lane < MAXC ? lane : 0] & 0xFF) - 1);
                const float lf = lamv / dt;
                L.dforce[d0] += L.cx[lane < MAXC ? lane : 0][0] * lf;
                L.dforce[d0 + 1] += L.cx[lane < MAXC ? lane : 0][1] * lf;
                L.dforce[d0 + 2] += L.cx[lane < MAXC ? lane : 0][2] * lf;
            }
            sync();
        } else {
        // ---- projected Gauss-Seidel over the rows (pgs_sweep): lane r keeps its unconstrained change,
        // its impulse and its bounds
        {
            const float invd = 1.0f / (act ? diag + 1e-12f : 1.f);
            // residual at the warm start: w = brow + A lambda0 (acol: lane c holds A[r][c] = A[c][r])
            float w0 = brow;
            if (__ballot(lam0 != 0.f)) {  // wave-uniform; rows >= nr hold no impulse
                auto aw = [&](auto nrows) {  // four independent accumulation chains, broadcasts in blocks of 4
                    constexpr int NRW = decltype(nrows)::value;
                    float wa[4] = {0.f, 0.f, 0.f, 0.f};
                    regla::static_for<0, NRW, 4>([&](auto rc) {
                        constexpr int r0 = decltype(rc)::value;
                        float sv[4];
                        regla::rdlane4<r0>(lam0, sv);
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (r0 + q < NRW) wa[(r0 + q) & 3] = fmaf(acol[r0 + q], sv[q], wa[(r0 + q) & 3]);
                    });
                    w0 += (wa[0] + wa[1]) + (wa[2] + wa[3]);
                };
                if (nr <= 16) aw(std::integral_constant<int, 16>{});
                else if (nr <= 32) aw(std::integral_constant<int, 32>{});
                else if (nr <= 48) aw(std::integral_constant<int, 48>{});
                else aw(std::integral_constant<int, MAXR>{});
            }
            lamv = lam0;
            float cd = act ? -w0 * invd : 0.f;
            const float ninvd = -invd;
            // the row's friction bound weight and its patch's normal rows n0 .. n0 + pc - 1 as a
            // 64-bit lane mask (friction rows only)
            const bool isn = kind == 0;
            const float muw = L.lam[lane];
            uint32_t mlo = 0u, mhi = 0u;
            if (act && !isn) {
                const int pc = rb1 == -1 ? L.tcnt[rb0] : 1;
                const uint64_t pm = ((1ull << pc) - 1ull) << (lane - (kind - 1) - pc);
                mlo = (uint32_t)pm;
                mhi = (uint32_t)(pm >> 32);
            }
            // a friction row's bound at the warm start: muw x its patch's normal impulses (<= 4 rows)
            float bnd = 0.f;
            if (__ballot(lam0 != 0.f)) {
                const int n0 = act && !isn ? (int)__builtin_ctzll(((uint64_t)mhi << 32) | mlo) : 0;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float v = __shfl(lam0, (n0 + j) & (W - 1), W);
                    const int bit = n0 + j;
                    const bool in = bit < 32 ? ((mlo >> (bit & 31)) & 1u) : ((mhi >> (bit & 31)) & 1u);
                    bnd += in ? v : 0.f;
                }
                bnd *= muw;
            }
            regla::f2v ak[MAXR];
            // the scaled columns acolp[r] = -A[r][lane] / A[lane][lane] and the packed bound weights of
            // the row-count class's rows only (the branch-free sweep reads no row past its class):
            // blocks of 16 rows, each behind a wave-uniform row-count test
            {
                const int nrb = __builtin_amdgcn_readfirstlane(nr);
                auto prep = [&](auto r0c) {
                    constexpr int R0 = decltype(r0c)::value;
#pragma unroll
                    for (int r = R0; r < (R0 + 16 < MAXR ? R0 + 16 : MAXR); ++r) {
                        const int sel = __builtin_amdgcn_sbfe((int)(r < 32 ? mlo : mhi), r & 31, 1);
                        ak[r] = regla::f2v{acol[r] * ninvd, __int_as_float(sel & __float_as_int(muw))};
                    }
                };
                prep(std::integral_constant<int, 0>{});
                if (nrb > 16) prep(std::integral_constant<int, 16>{});
                if (nrb > 32) prep(std::integral_constant<int, 32>{});
                if (nrb > 48) prep(std::integral_constant<int, 48>{});
            }
            const float kInf = __builtin_inff();
            float lo = isn ? -lamv : -bnd - lamv;
            float hi = isn ? kInf : bnd - lamv;
            const int nru = __builtin_amdgcn_readfirstlane(nr);
            STAMP(22);  // the solve's set-up (warm-start residual, bounds, scaled columns) apart from its sweeps
            __builtin_amdgcn_s_setprio(kPrioSerial);
            const float tol = p.solver_tolerance;
            for (int it = 0; it < p.solver_iterations; ++it) {
                float dvec = 0.f;
                // the row count through an opaque copy per sweep: the 63 early-exit compares stay
                // scalar compares in the sweep instead of being hoisted out of the loop as 63
                // lane-mask pairs (SGPR spills)
                int nrs = nru;
                asm volatile("" : "+s"(nrs));
                regla::f2v ch = {cd, hi};
                if (nrs <= 16) pgs_sweep_fix<0, 16>(ch, dvec, lo, ak, nrs);
                else
                if (nrs <= 32) pgs_sweep_fix<0, 32>(ch, dvec, lo, ak, nrs);
                else if (nrs <= 48) pgs_sweep_fix<0, 48>(ch, dvec, lo, ak, nrs);
                else pgs_sweep_fix<0, MAXR>(ch, dvec, lo, ak, nrs);
                cd = ch.x;
                hi = ch.y;
                // the bound at the sweep's end: B = hi + lambda(start); then the bounds about the new impulse
                const float bn = hi + lamv;
                lamv += dvec;
                lo = isn ? -lamv : -bn - lamv;
                hi = isn ? kInf : bn - lamv;
                // converged (optional, solver_tolerance > 0): no row's velocity moved by more than
                // the tolerance in this sweep, |d lambda_r| A_rr (oracle: the same test)
                if (tol > 0.f && __ballot(act && fabsf(dvec) * diag > tol) == 0ull) break;
            }
            __builtin_amdgcn_s_setprio(kPrioDefault);
        }
        // the solve's impulses and row keys: the next solve's warm start and the reported forces
        L.lam[lane] = act ? lamv : 0.f;
        if (lane == 0) L.nwc = p.warm_start ? nr : 0;  // warm_start 0: every substep's solve is cold
        sync();
        STAMP(10);
        // ---- du = M^-1 J^T lambda = L^-1 D^-1/2 (Zh^T lambda): lane r scales its row by lambda_r,
        // a wave reduce-scatter sums the 75 columns into lane = dof, then one L^-1 sweep
        {
            __builtin_amdgcn_s_setprio(kPrioDefault);
            float v64[64], v16[16];
#pragma unroll
            for (int i = 0; i < 64; ++i) v64[i] = ZV(z, i) * lamv;
#pragma unroll
            for (int i = 0; i < 16; ++i) v16[i] = 64 + i < NG ? ZV(z, 64 + i < NG ? 64 + i : 0) * lamv : 0.f;
            float yl = reduce_scatter<64>(v64);
            float y2 = __shfl(reduce_scatter<16>(v16), 4 * (lane & 15), W);
            yl = (yl + L.yh[lane]) * L.sDinv[lane];
            y2 = lane < NH ? (y2 + L.yh[64 + lane]) * L.sDinv[64 + lane] : 0.f;
            float r1[regla::kRowRegs], r2[regla::kRowRegs];
            load_rows(L, T, lane, r1, r2);
            solve_L(r1, r2, lane, yl, y2);
            __builtin_amdgcn_s_setprio(kPrioDefault);
            L.uf[lane] = L.u0[lane] + yl;
            if (lane < NH) L.uf[64 + lane] = L.u0[64 + lane] + y2;
        }
        }  // PGS
        // ---- reported contact forces (net linear contact impulse per body / dt): the output is the
        // last substep's, so the earlier substeps skip them (their cf rows stay zero, as set above)
        if (last) {
            float* fr = gl + 2 * kCand;  // per-row linear impulses: the stored directions x lambda
            if (act) {
                fr[3 * lane] *= lamv;
                fr[3 * lane + 1] *= lamv;
                fr[3 * lane + 2] *= lamv;
            }
            sync();
            if (lane < NB) {
                // the body's own terrain rows (its patch: a contiguous row range, in row order), then
                // the self-pair rows with their sign; the same summation order as over all rows
                float F3[3] = {0.f, 0.f, 0.f};
                const int tn = L.tcnt[lane];
                const int r0 = tn > 0 ? L.srow0[L.tbase[lane]] : 0;
                const int rn = tn == 0 ? 0 : tn + (tn >= 2 ? 3 : 2);
#pragma unroll
                for (int k = 0; k < 7; ++k) {
                    if (k < rn) {
                        const int r = r0 + k;
                        for (int x = 0; x < 3; ++x) F3[x] += fr[3 * r + x];
                    }
                }
                const int nterr = __builtin_amdgcn_readfirstlane(L.nterr);
                for (int c = nterr; c < nc; ++c) {  // wave-uniform bounds
                    const int cb = L.cbb[c];
                    const float sg = ((cb & 0xFF) == lane ? 1.f : 0.f) - ((cb >> 8) - 2 == lane ? 1.f : 0.f);
                    const int r = L.srow0[c];
                    for (int k = 0; k < 3; ++k)
                        for (int x = 0; x < 3; ++x) F3[x] += sg * fr[3 * (r + k) + x];
                }
                L.cf[lane][0] = F3[0] / dt; L.cf[lane][1] = F3[1] / dt; L.cf[lane][2] = F3[2] / dt;
            }
            sync();
        }  // last
    }
    if (nr == 0) {  // nothing to warm-start the next solve from
        L.lam[lane] = 0.f;
        if (lane == 0) L.nwc = 0;
    }
    if (TGS && nr == 0) {  // TGS without contact rows: the iterations' drives and bias only
        for (int it = 0; it < K; ++it) {
            tgs_velocity(L, T, lane, 0.f, 0.f);
            STAMP(11);
            tgs_advance(it);
        }
        tgs_drive_out();
    }
    if (!TGS && nr == 0) {  // no contact: uf = u0 + L^-1 D^-1/2 yh
        float yl = L.yh[lane] * L.sDinv[lane];
        float y2 = lane < NH ? L.yh[64 + lane] * L.sDinv[64 + lane] : 0.f;
        float r1[regla::kRowRegs], r2[regla::kRowRegs];
        load_rows(L, T, lane, r1, r2);
        solve_L(r1, r2, lane, yl, y2);
        L.uf[lane] = L.u0[lane] + yl;
        if (lane < NH) L.uf[64 + lane] = L.u0[64 + lane] + y2;
        sync();
    }
    STAMP(11);
    if constexpr (TGS) {  // TGS: the iterations integrated the positions and set the drive force
        STAMP(12);
        return;
    }
    // ---- drive force actually applied, damping, clamps, write velocities
    if (last) {  // the reported drive force is the last substep's
        for (int i = lane; i < NG; i += W)
            if (i >= 6) L.dforce[i - 6] -= L.coef[i] * (L.uf[i] - L.u0[i]);
        sync();
        // plus the joint-limit force (dof_force = the joint's solver force, drive and limit together;
        // oracle/he_oracle_physics.c): limit slot c (one per joint, row c) adds g lambda / dt over its
        // joint's dofs, g = its row (kept in the contact-position words)
        const int nl = __builtin_amdgcn_readfirstlane(L.nlim);
        if (lane < nl && nr > 0) {
            const int d0 = 3 * ((L.cbb[lane < MAXC ? lane : 0] & 0xFF) - 1);
            const float lf = L.lam[lane] / dt;
            L.dforce[d0] += L.cx[lane < MAXC ? lane : 0][0] * lf;
            L.dforce[d0 + 1] += L.cx[lane < MAXC ? lane : 0][1] * lf;
            L.dforce[d0 + 2] += L.cx[lane < MAXC ? lane : 0][2] * lf;
        }
        sync();
    }
    integrate_bodies(L, T, lane, p, dt, damp, L.uf, true, !last);
    STAMP(12);
}

// two waves per SIMD need at most 256 VGPRs + AGPRs. Unbounded, the allocator lands at 257 (one
// kernel-lifetime value parked in an AGPR) and the kernel falls to one wave per SIMD; the bound
// makes it fit without scratch. humanoid_amd/build.py checks the compiler's occupancy report and
// fails the build below 2 waves per SIMD either way. (Round 3 A/B, profiles/r03/ab_lt_pipe.txt:
// the pipelined midpoint L^-T with the bound +3.0 % against the grouped one without it, which
// fits in 251 unbounded.)
#ifndef HE_MIN_WAVES
#define HE_MIN_WAVES 2
#endif
template <bool TGS>
HE_DEV void physics_body(const PhysArgs& a) {
    extern __shared__ float smem[];
    Lds& L = *reinterpret_cast<Lds*>(smem);
    if ((int)blockIdx.x >= a.num_envs) return;  // the first-dispatch warm-up (warm_physics_kernels): no env
    const int lane = threadIdx.x;
    // the env of this workgroup (launch_physics_order: heavy envs first); it and the start cycle wait
    // in LDS for the epilogue (no registers held through the substeps)
    // The order is rebuilt on the launch stream (he_engine.cpp); an index outside [0, num_envs) (a
    // stray write into the buffer) falls back to workgroup id = env instead of faulting.
    int e0 = a.order ? a.order[blockIdx.x] : (int)blockIdx.x;
    if ((unsigned)e0 >= (unsigned)a.num_envs) e0 = (int)blockIdx.x;
    int e = e0;
    if (lane == 0) {
        L.sch_t0 = __builtin_readcyclecounter();
        L.sch_e = e0;
    }
    const he_model& m = *a.model;
    // ---- body-level tree tables into LDS
    if (lane < NB) {
        const PhysTopo& T = *a.topo;
        L.T.depth[lane] = T.body_depth[lane];
        for (int k = 0; k < 9; ++k) L.T.chain[lane][k] = T.body_chain[lane][k];
        L.T.dof0[lane] = T.body_dof0[lane];
        L.T.anc_mask[lane] = T.anc_mask[lane];
        L.T.sub_mask[lane] = T.sub_mask[lane];
        L.T.jump4[lane] = kJump4.v[lane < NB ? lane : 0];
        for (int c = 0; c < 3; ++c) L.T.local_pos[lane][c] = m.local_pos[lane][c];
    }
    L.T.cbody[lane] = a.topo->corner_body[lane];
    for (int i = lane; i < NG; i += W) {  // per-dof tree tables (constant memory -> LDS once)
        L.T.pack_start[i] = (int16_t)smpl::kPackStart[i];
        L.T.dof_depth[i] = (int8_t)(smpl::kDofNanc[i] - 1);
    }
    // ---- load state
    const float* rs = a.root_states + (size_t)e * 13;
    if (lane < 3) { L.root_pos[lane] = rs[lane]; L.u0[3 + lane] = rs[7 + lane]; L.u0[lane] = rs[10 + lane]; }
    if (lane < 4) L.root_q[lane] = rs[3 + lane];
    for (int d = lane; d < ND; d += W) {
        L.q[d] = a.dof_state[((size_t)e * ND + d) * 2];
        L.u0[6 + d] = a.dof_state[((size_t)e * ND + d) * 2 + 1];
        float t;
        if (a.actions) {  // humanoid_phc.py:1218-1228 + freeze :116-125
            float act = a.actions[(size_t)e * ND + d];
            if (a.clip_actions) act = fminf(fmaxf(act, -1.f), 1.f);
            t = a.frozen[d] ? 0.f : a.pd_offset[d] + a.pd_scale[d] * act;
            a.dof_targets[(size_t)e * ND + d] = t;
        } else {
            t = a.dof_targets[(size_t)e * ND + d];
        }
        L.tgt[d] = t;
    }
    // ---- warm-start cache (include/humanoid_engine.h HE_CACHE_WORDS): valid while the root pose
    // still equals the signature the previous step wrote (an external write -- a reset -- breaks it)
    {
        const float* cw = a.cache ? a.cache + (size_t)e * HE_CACHE_WORDS : nullptr;
        const float w1 = cw ? cw[lane] : 0.f;
        const float w2 = cw && lane < HE_CACHE_WORDS - W ? cw[W + (lane < HE_CACHE_WORDS - W ? lane : 0)] : 0.f;
        const float sig = lane < 3 ? rs[lane] : (lane < 7 ? rs[lane < 7 ? lane : 0] : 0.f);
        const bool diff = lane < 7 && __float_as_uint(w1) != __float_as_uint(sig);
        const bool valid = cw && a.p.warm_start && __ballot(diff) == 0ull;
        const int nw = valid ? __builtin_amdgcn_readlane(__float_as_int(w1), 7) : 0;
        const int nwc = nw < 0 ? 0 : (nw > MAXR ? MAXR : nw);
        // row keys: 16 bits each, rows 2j / 2j + 1 in word HE_CACHE_KEYS + j
        constexpr int KW = (MAXR + 1) / 2;
        if (lane >= HE_CACHE_KEYS && lane < HE_CACHE_KEYS + KW) {
            const int j = lane - HE_CACHE_KEYS;
            const uint32_t kw = __float_as_uint(w1);
            L.wckey[2 * j] = (int)(kw & 0xFFFFu);
            L.wckey[2 * j + 1] = (int)(kw >> 16);
        }
        // impulses: rows 0 .. W - HE_CACHE_LAMBDA - 1 from the first read, the rest from the second
        if (lane >= HE_CACHE_LAMBDA) L.lam[lane - HE_CACHE_LAMBDA] = valid ? w1 : 0.f;
        if (lane < HE_CACHE_LAMBDA) L.lam[W - HE_CACHE_LAMBDA + lane] = valid && W + lane < HE_CACHE_WORDS ? w2 : 0.f;
        if (lane == 0) L.nwc = nwc;
    }
    static_assert(HE_CACHE_KEYS + (MAXR + 1) / 2 <= HE_CACHE_LAMBDA && HE_CACHE_LAMBDA + MAXR <= HE_CACHE_WORDS &&
                  HE_CACHE_WORDS <= 2 * W && HE_CACHE_LAMBDA < W, "cache layout");
    if (a.fused && lane == 0) {  // fused imitation: bookkeeping + motion metadata (trips 1, 2) now
        const ImitArgs& im = a.im;
        const int64_t mid = clamp_mid(im.m, im.motion_ids[e]);
        const ImitBook bk = imitation_book(im, mid, f3{im.global_offset[3 * e], im.global_offset[3 * e + 1],
                                                       im.global_offset[3 * e + 2]},
                                           im.start_times[e], im.start_offsets[e], im.progress[e]);
        __builtin_memcpy(L.imbook, &bk, sizeof(ImitBook));
    }
    sync();
    if (a.p.joint_limits) {  // the first substep's limit rows, from the loaded state
        const bool joint = lane >= 1 && lane < NB;
        const int d = 3 * (joint ? lane - 1 : 0);
        limit_detect(L, lane, joint, f3{L.q[d], L.q[d + 1], L.q[d + 2]}, f3{L.u0[6 + d], L.u0[7 + d], L.u0[8 + d]}, a.p);
        sync();
    }
    const float* ms = a.mass_scale ? a.mass_scale + (size_t)e * NB : nullptr;
    float mu = a.friction ? a.friction[e] : a.p.friction;
    int tk = (a.p.terrain && a.terrain_kind) ? a.terrain_kind[e] : 0;
    unsigned long long* stamps = a.stamps ? a.stamps + (size_t)e * HE_STAMP_SLOTS : nullptr;
    unsigned long long t_prev = __builtin_readcyclecounter();
    for (int s = 0; s < a.substeps; ++s)
        substep<TGS>(L, a, a.model, lane, ms, mu, tk, stamps, t_prev, s == 0, s == a.substeps - 1);
    // ---- fused imitation (he_env_step): the reference samples depend only on the env's motion
    // bookkeeping (read into LDS at the kernel's start), so their loads are issued here and land
    // behind the final kinematics and stores
    ImitRaw iraw;
    if (a.fused && lane < GROUP) {
        ImitBook bk;
        static_assert(sizeof(ImitBook) <= sizeof(L.imbook), "ImitBook fits its LDS words");
        __builtin_memcpy(&bk, L.imbook, sizeof(ImitBook));
        iraw = imitation_frames_load(a.im, lane, bk);  // loads only: the blends wait for the epilogue
    }
    // ---- outputs: generalized state, FK rigid-body state, forces
    e = L.sch_e;  // from LDS: not held through the substeps
    kinematics<false>(L, m, lane, a.p, a.substeps > 0);
    STAMP(13);
    float* rso = a.root_states + (size_t)e * 13;
    if (lane < 3) { rso[lane] = L.root_pos[lane]; rso[7 + lane] = L.u0[3 + lane]; rso[10 + lane] = L.u0[lane]; }
    if (lane < 4) rso[3 + lane] = L.root_q[lane];
    for (int d = lane; d < ND; d += W) {
        a.dof_state[((size_t)e * ND + d) * 2] = L.q[d];
        a.dof_state[((size_t)e * ND + d) * 2 + 1] = L.u0[6 + d];
        a.dof_force[(size_t)e * ND + d] = L.dforce[d];
    }
    // rigid-body rows, lane = body (the fused epilogue reads its body from the same registers)
    SimBody sb = body_row(L, lane < NB ? lane : 0);
    if (lane < NB) {
        float* rb = a.rb_state + ((size_t)e * NB + lane) * 13;
        rb[0] = sb.pos.x; rb[1] = sb.pos.y; rb[2] = sb.pos.z;
        rb[3] = sb.rot.x; rb[4] = sb.rot.y; rb[5] = sb.rot.z; rb[6] = sb.rot.w;
        rb[7] = sb.vel.x; rb[8] = sb.vel.y; rb[9] = sb.vel.z;
        rb[10] = sb.ang.x; rb[11] = sb.ang.y; rb[12] = sb.ang.z;
    }
    for (int t = lane; t < NB * 3; t += W) a.contact_forces[(size_t)e * NB * 3 + t] = L.cf[t / 3][t % 3];
    if (lane == 0 && a.num_contacts) a.num_contacts[e] = L.nc;
    if (lane == 0 && a.dropped) a.dropped[e] = L.ncand - L.nc;
    if (a.fused && lane < GROUP) {
        // he_env_step: the imitation step of this env on lanes 0..31 (lane = body), after every
        // physics store above has landed (a fused reset overwrites those rows)
        __threadfence_block();
        float pw = 0.0f;
        if (a.im.p.use_power_reward && lane < NB - 1)  // the joint's |tau . qdot| (humanoid_phc.py:1297-1305)
            pw = power_term(&L.dforce[3 * lane], &L.u0[6 + 3 * lane], 1);
        imitation_finish<false>(a.im, e, e, lane, lane == 0, imitation_frames_blend(iraw), sb, pw);
    }
    STAMP(24);
    if (a.cache) {  // signature (the root pose just written), row count, row keys, impulses
        float* cw = a.cache + (size_t)e * HE_CACHE_WORDS;
        const int nwc = a.p.warm_start ? L.nwc : 0;
        constexpr int KW = (MAXR + 1) / 2;
        float v = 0.f;
        if (lane < 3) v = L.root_pos[lane];
        else if (lane < 7) v = L.root_q[lane < 7 ? lane - 3 : 0];
        else if (lane == 7) v = __int_as_float(nwc);
        else if (lane < HE_CACHE_KEYS + KW) {
            const int j = lane - HE_CACHE_KEYS;
            const uint32_t k0 = 2 * j < nwc ? (uint32_t)L.wckey[2 * j] & 0xFFFFu : 0u;
            const uint32_t k1 = 2 * j + 1 < nwc ? (uint32_t)L.wckey[2 * j + 1] & 0xFFFFu : 0u;
            v = __uint_as_float(k0 | (k1 << 16));
        } else if (lane >= HE_CACHE_LAMBDA) v = lane - HE_CACHE_LAMBDA < nwc ? L.lam[lane - HE_CACHE_LAMBDA] : 0.f;
        if (!a.p.warm_start) v = 0.f;
        cw[lane] = v;
        if (lane < HE_CACHE_WORDS - W) {
            const int r = W - HE_CACHE_LAMBDA + lane;
            cw[W + lane] = a.p.warm_start && r < nwc ? L.lam[r] : 0.f;
        }
    }
    if (a.cost && lane == 0) {  // this env's cycles, for the next launch's order
        const unsigned long long cyc = __builtin_readcyclecounter() - L.sch_t0;
        a.cost[e] = cyc > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)cyc;
    }
}

// he_sim_params.solver_type 0 (PGS) and 1 (TGS): one instantiation each, so that the TGS iterations'
// register plan does not touch the PGS kernel's
__global__ void __launch_bounds__(64, HE_MIN_WAVES) physics_kernel(PhysArgs a) { physics_body<false>(a); }
__global__ void __launch_bounds__(64, HE_MIN_WAVES) physics_kernel_tgs(PhysArgs a) { physics_body<true>(a); }

}  // namespace

static_assert(sizeof(Lds) <= 20480, "two workgroups per SIMD (8 per CU) need <= 20 KB of LDS each");
#ifndef HE_LDS_EXTRA  // diagnostics only: extra dynamic LDS per wave, to run fewer waves per CU
#define HE_LDS_EXTRA 0   // (one wave alone on its CU; round 4)
#endif
size_t physics_lds_bytes() { return (sizeof(Lds) + 15) / 16 * 16 + HE_LDS_EXTRA; }

bool physics_phase_stamps() { return HE_PHASE_STAMPS != 0; }

namespace {
// launch_physics_order (he_kernels.h): one workgroup of 1024 threads (16 waves). The mean cost, then
// each env's class by its cost relative to the mean, kOrderClasses classes of mean / 32 from
// 0.5 x mean to 1.5 x mean (outside: the end classes; order_class), and order[] partitioned by
// class, the costliest class first: a longest-first order in steps of ~3 % of the mean. One pass
// sizes the classes, the second places every env after the costlier classes (order_wave).
constexpr int kOrderThreads = 1024;
constexpr int kOrderWaves = kOrderThreads / 64;
constexpr int kOrderClasses = 32;
// floor(32 c / mean) - 16 clamped to the classes, in integers (the host restates it exactly:
// tests/test_full_size.py): class >= m exactly when c >= T[m] = ceil((m + 16) tot / (32 n)), so the
// class is found by a binary search over the 31 thresholds (one 64-bit division per threshold, not
// per env)
__device__ __forceinline__ int order_class(uint32_t c, const uint32_t* thr) {
    int lo = 0;  // the largest m with c >= thr[m] (thr[0] = 0)
#pragma unroll
    for (int step = 16; step > 0; step >>= 1)
        if (lo + step < kOrderClasses && c >= thr[lo + step]) lo += step;
    return lo;
}
// Each wave takes the classes of its lanes' kOrderPer envs (env r0 + 1024 j + 64 w + lane, j <
// kOrderPer) one distinct class at a time (the first remaining element's class): the class's
// elements rank themselves by its ballots, and one lane adds their count to the class's LDS cursor
// (an atomic per distinct class and wave, not per env). The cursor's order between waves is the
// atomics', so envs of one class are not in env order; results do not depend on the order (envs
// never interact).
constexpr int kOrderPer = 4;
__device__ __forceinline__ void order_wave(const int (&k)[kOrderPer], int lane, int* cursor, int (&slot)[kOrderPer]) {
    const unsigned long long lt = (1ull << lane) - 1ull;
    unsigned long long left[kOrderPer];
#pragma unroll
    for (int j = 0; j < kOrderPer; ++j) left[j] = __ballot(k[j] >= 0);
    for (;;) {
        int j0 = -1;
#pragma unroll
        for (int j = kOrderPer - 1; j >= 0; --j) j0 = left[j] ? j : j0;
        if (j0 < 0) break;
        int kc = 0;
#pragma unroll
        for (int j = 0; j < kOrderPer; ++j)
            if (j == j0) kc = __shfl(k[j], __builtin_ctzll(left[j]), 64);
        unsigned long long m[kOrderPer];
        int cnt = 0, before[kOrderPer];
#pragma unroll
        for (int j = 0; j < kOrderPer; ++j) {
            m[j] = __ballot(k[j] == kc);
            before[j] = cnt;
            cnt += __popcll(m[j]);
            left[j] &= ~m[j];
        }
        int b = 0;
        if (lane == 0) b = atomicAdd(&cursor[kc], cnt);
        b = __shfl(b, 0, 64);
#pragma unroll
        for (int j = 0; j < kOrderPer; ++j)
            if (k[j] == kc) slot[j] = b + before[j] + __popcll(m[j] & lt);
    }
}
__global__ void __launch_bounds__(kOrderThreads) physics_order_kernel(const uint32_t* cost, int32_t* order, int n) {
    __shared__ unsigned long long red[kOrderWaves];
    __shared__ int hist[kOrderClasses], cursor[kOrderClasses];
    __shared__ uint32_t thr[kOrderClasses];
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    unsigned long long s = 0;
    for (int i = t; i < n; i += kOrderThreads) s += cost[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if (lane == 0) red[w] = s;
    if (t < kOrderClasses) hist[t] = 0;
    __syncthreads();
    if (t < kOrderClasses) {
        unsigned long long tot = 0;
        for (int v = 0; v < kOrderWaves; ++v) tot += red[v];
        const unsigned long long d = 32ull * (unsigned long long)(n > 0 ? n : 1);
        const unsigned long long x = (unsigned long long)(t + 16) * tot;
        const unsigned long long T = t == 0 ? 0ull : (x + d - 1) / d;
        thr[t] = T > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)T;
    }
    __syncthreads();
    int k[kOrderPer], slot[kOrderPer];
    auto classes = [&](int r0) {
#pragma unroll
        for (int j = 0; j < kOrderPer; ++j) {
            const int e = r0 + kOrderThreads * j + t;
            k[j] = e < n ? order_class(cost[e], thr) : -1;
        }
    };
    for (int r0 = 0; r0 < n; r0 += kOrderPer * kOrderThreads) {  // the classes' sizes
        classes(r0);
        order_wave(k, lane, hist, slot);
    }
    __syncthreads();
    if (t == 0) {  // the costliest class first
        int acc = 0;
        for (int c = kOrderClasses - 1; c >= 0; --c) { cursor[c] = acc; acc += hist[c]; }
    }
    __syncthreads();
    for (int r0 = 0; r0 < n; r0 += kOrderPer * kOrderThreads) {
        classes(r0);
        order_wave(k, lane, cursor, slot);
#pragma unroll
        for (int j = 0; j < kOrderPer; ++j)
            if (k[j] >= 0) order[slot[j]] = r0 + kOrderThreads * j + t;
    }
}
}  // namespace

namespace {
__global__ void warm_tu_kernel() {}
}  // namespace

#define HE_RETURN_IF(x)                      \
    do {                                     \
        const hipError_t e_ = (x);           \
        if (e_ != hipSuccess) return e_;     \
    } while (0)
hipError_t warm_physics_kernels(hipStream_t stream, int mode) {
    if (mode == 1) {
        warm_tu_kernel<<<1, 64, 0, stream>>>();
        return hipGetLastError();
    }
    PhysArgs pa{};
    physics_kernel<<<1, W, physics_lds_bytes(), stream>>>(pa);
    HE_RETURN_IF(hipGetLastError());
    physics_kernel_tgs<<<1, W, physics_lds_bytes(), stream>>>(pa);
    HE_RETURN_IF(hipGetLastError());
    physics_order_kernel<<<1, kOrderThreads, 0, stream>>>(nullptr, nullptr, 0);
    return hipGetLastError();
}


hipError_t launch_physics_order(const uint32_t* cost, int32_t* order, int num_envs, hipStream_t stream) {
    if (num_envs <= 0) return hipSuccess;
    physics_order_kernel<<<1, kOrderThreads, 0, stream>>>(cost, order, num_envs);
    return hipGetLastError();
}

hipError_t launch_physics(const PhysArgs& a, hipStream_t stream) {
    if (a.num_envs <= 0) return hipSuccess;
    const size_t lds = physics_lds_bytes();
    if (a.p.solver_type == 1) physics_kernel_tgs<<<a.num_envs, W, lds, stream>>>(a);
    else physics_kernel<<<a.num_envs, W, lds, stream>>>(a);
    return hipGetLastError();
}
