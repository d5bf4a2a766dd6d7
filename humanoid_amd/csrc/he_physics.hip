// he_physics.hip -- articulated SMPL-humanoid step for gfx950 (replaces
// gym.simulate x control_freq_inv, puffer_phc/envs/humanoid_phc.py:131-134).
//
// Mapping: one environment per 64-lane workgroup (one wave), all substeps of a policy step in
// one launch. Generalized state lives in LDS for the whole launch; HBM sees one coalesced read of
// the env's root/dof/target rows and one write of root/dof/rigid-body/contact/dof-force rows.
// Lanes parallelise over bodies (24), dofs (75), sparse mass-matrix entries (1221), contact
// rows (3 x contacts) and elimination pairs; the tree-ordered sweeps are expressed through static
// root-first chain tables (he_topo.h) so each lane walks its own chain without waiting on levels.
//
// Algorithm (DESIGN.md §3, fp64 reference oracle/he_oracle_physics.c):
//   FK -> spatial axes S about the root origin -> RNEA bias -> CRBA (+armature) -> implicit PD
//   -> sparse LTDL -> free velocity -> ground/self contacts -> Z = L^-T J^T, A = Z^T D^-1 Z
//   -> PGS (residuals kept in registers, one LDS column read per row update) -> velocity update
//   -> damping / clamps -> semi-implicit integration.
#include <hip/hip_runtime.h>

#include "../../include/humanoid_engine.h"
#include "he_kernels.h"
#include "he_math.h"
#include "he_topo.h"

namespace {

constexpr int NB = HE_NUM_BODIES;
constexpr int ND = HE_NUM_DOF;
constexpr int NG = HE_NUM_GEN;
constexpr int MAXC = HE_MAX_CONTACTS;
constexpr int W = 64;

struct Lds {
    float q[ND], tgt[ND];
    float u0[NG], uf[NG], y[NG], coef[NG], rhs[NG];
    float ql[NB][4], qw[NB][4], pw[NB][3];
    float S[NG][6], IS[NG][6];
    float V[NB][6], Acc[NB][6], F[NB][6];
    float Ib[NB][10], Ic[NB][10];  // m, h(3), I(xx yy zz xy xz yz)
    float H[HE_NNZ_MAX];
    float cx[MAXC][3], cn[MAXC][3], ct1[MAXC][3], ct2[MAXC][3], cgap[MAXC], cmu[MAXC];
    int cb0[MAXC], cb1[MAXC];
    float brow[3 * MAXC];
    float cf[NB][3];
    float dforce[ND];
    float Dinv[NG];
    float root_pos[3], root_q[4];
    int nc;
    PhysTopo T;  // static tables copied from global memory once per launch
};

HE_DEV void sync() { __syncthreads(); }

// optional per-phase cycle stamps (diagnostic: PhysArgs.stamps != null), lane 0 accumulates
// s_memtime deltas per phase into stamps[block * 16 + phase]
#define STAMP(id)                                                             \
    do {                                                                      \
        if (stamps && lane == 0) {                                            \
            unsigned long long _t = __builtin_readcyclecounter();             \
            stamps[id] += _t - t_prev;                                        \
            t_prev = _t;                                                      \
        }                                                                     \
    } while (0)

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

HE_DEV f3 body_point(const Lds& L, int b, f3 local) {
    f4 q = f4{L.qw[b][0], L.qw[b][1], L.qw[b][2], L.qw[b][3]};
    return f3{L.pw[b][0], L.pw[b][1], L.pw[b][2]} + qapply(q, local);
}

HE_DEV float terrain_dist(const he_sim_params& p, int kind, f3 x, f3& n) {
    if (kind == 1) {
        float s = sinf(p.terrain_slope), c = cosf(p.terrain_slope);
        n = f3{-s, 0.f, c};
        return dot3(n, x);
    }
    n = f3{0.f, 0.f, 1.f};
    if (kind == 2) {
        float h = x.x > 0.f ? p.step_height * floorf(x.x / p.step_length) : 0.f;
        return x.z - h;
    }
    return x.z;
}

HE_DEV void body_segment(const he_model& m, const Lds& L, int b, f3& a, f3& c, float& r) {
    const float* g = m.geom_params[b];
    int gt = m.geom_type[b];
    if (gt == HE_GEOM_SPHERE) {
        a = body_point(L, b, f3{g[0], g[1], g[2]});
        c = a;
        r = g[3];
    } else if (gt == HE_GEOM_CAPSULE) {
        a = body_point(L, b, f3{g[0], g[1], g[2]});
        c = body_point(L, b, f3{g[3], g[4], g[5]});
        r = g[6];
    } else {
        float e[3] = {g[3], g[4], g[5]};
        int ax = 0;
        if (e[1] > e[ax]) ax = 1;
        if (e[2] > e[ax]) ax = 2;
        float rp = m.geom_radius[b];
        float half = fmaxf(e[ax] - rp, 0.f);
        f4 bq = f4{g[6], g[7], g[8], g[9]};
        f3 unit = ax == 0 ? f3{1.f, 0.f, 0.f} : (ax == 1 ? f3{0.f, 1.f, 0.f} : f3{0.f, 0.f, 1.f});
        f3 dir = qapply(bq, unit) * half;
        f3 ctr = f3{g[0], g[1], g[2]};
        a = body_point(L, b, ctr - dir);
        c = body_point(L, b, ctr + dir);
        r = rp;
    }
}

// closest points between segments p1q1 and p2q2 (Ericson, RTCD 5.1.9)
HE_DEV void seg_seg(f3 p1, f3 q1, f3 p2, f3 q2, f3& c1, f3& c2) {
    f3 d1 = q1 - p1, d2 = q2 - p2, r = p1 - p2;
    float a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    float s, t;
    const float eps = 1e-12f;
    if (a <= eps && e <= eps) { s = t = 0.f; }
    else if (a <= eps) { s = 0.f; t = fminf(fmaxf(f / e, 0.f), 1.f); }
    else {
        float c = dot3(d1, r);
        if (e <= eps) { t = 0.f; s = fminf(fmaxf(-c / a, 0.f), 1.f); }
        else {
            float b = dot3(d1, d2), den = a * e - b * b;
            s = den > eps ? fminf(fmaxf((b * f - c * e) / den, 0.f), 1.f) : 0.f;
            t = (b * s + f) / e;
            if (t < 0.f) { t = 0.f; s = fminf(fmaxf(-c / a, 0.f), 1.f); }
            else if (t > 1.f) { t = 1.f; s = fminf(fmaxf((b - c) / a, 0.f), 1.f); }
        }
    }
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

// wave-wide exclusive prefix count of `flag` (uint64 ballot)
HE_DEV int wave_prefix(bool flag, int lane, int& total) {
    uint64_t m = __ballot(flag);
    total = __popcll(m);
    uint64_t below = lane == 0 ? 0ull : (m & ((~0ull) >> (64 - lane)));
    return __popcll(below);
}

HE_DEV void store_contact(Lds& L, int slot, int b0, int b1, f3 x, f3 n, float gap, float mu) {
    L.cb0[slot] = b0;
    L.cb1[slot] = b1;
    L.cx[slot][0] = x.x; L.cx[slot][1] = x.y; L.cx[slot][2] = x.z;
    L.cn[slot][0] = n.x; L.cn[slot][1] = n.y; L.cn[slot][2] = n.z;
    f3 t1, t2;
    friction_basis(n, t1, t2);
    L.ct1[slot][0] = t1.x; L.ct1[slot][1] = t1.y; L.ct1[slot][2] = t1.z;
    L.ct2[slot][0] = t2.x; L.ct2[slot][1] = t2.y; L.ct2[slot][2] = t2.z;
    L.cgap[slot] = gap;
    L.cmu[slot] = mu;
}

// ---------------------------------------------------------------------------------- kinematics
HE_DEV void kinematics(Lds& L, const he_model& m, const PhysTopo& T, int lane) {
    if (lane < NB) {
        if (lane == 0) {
            L.ql[0][0] = L.root_q[0]; L.ql[0][1] = L.root_q[1]; L.ql[0][2] = L.root_q[2]; L.ql[0][3] = L.root_q[3];
        } else {
            int d = 3 * (lane - 1);
            f4 q = qexp(f3{L.q[d], L.q[d + 1], L.q[d + 2]});
            L.ql[lane][0] = q.x; L.ql[lane][1] = q.y; L.ql[lane][2] = q.z; L.ql[lane][3] = q.w;
        }
    }
    sync();
    if (lane < NB) {
        // walk this body's chain from the root
        f4 q = qnormalize(f4{L.ql[0][0], L.ql[0][1], L.ql[0][2], L.ql[0][3]});
        f3 p = f3{L.root_pos[0], L.root_pos[1], L.root_pos[2]};
        int depth = T.body_depth[lane];
        for (int k = 1; k <= depth; ++k) {
            int a = T.body_chain[lane][k];
            p = p + qapply(q, f3{m.local_pos[a][0], m.local_pos[a][1], m.local_pos[a][2]});
            q = qmul(q, f4{L.ql[a][0], L.ql[a][1], L.ql[a][2], L.ql[a][3]});
        }
        L.qw[lane][0] = q.x; L.qw[lane][1] = q.y; L.qw[lane][2] = q.z; L.qw[lane][3] = q.w;
        L.pw[lane][0] = p.x; L.pw[lane][1] = p.y; L.pw[lane][2] = p.z;
    }
    sync();
    f3 o = f3{L.root_pos[0], L.root_pos[1], L.root_pos[2]};
    for (int i = lane; i < NG; i += W) {
        float* S = L.S[i];
        if (i < 6) {
            for (int c = 0; c < 6; ++c) S[c] = (c == i) ? 1.f : 0.f;
        } else {
            int b = T.dof_body[i], c = (i - 6) % 3;
            f4 q = f4{L.qw[b][0], L.qw[b][1], L.qw[b][2], L.qw[b][3]};
            f3 e = c == 0 ? f3{1.f, 0.f, 0.f} : (c == 1 ? f3{0.f, 1.f, 0.f} : f3{0.f, 0.f, 1.f});
            f3 a = qapply(q, e);
            f3 l = cross3(f3{L.pw[b][0], L.pw[b][1], L.pw[b][2]} - o, a);
            S[0] = a.x; S[1] = a.y; S[2] = a.z; S[3] = l.x; S[4] = l.y; S[5] = l.z;
        }
    }
    sync();
    if (lane < NB) {
        float V[6] = {L.u0[0], L.u0[1], L.u0[2], L.u0[3], L.u0[4], L.u0[5]};
        int depth = T.body_depth[lane];
        for (int k = 1; k <= depth; ++k) {
            int a = T.body_chain[lane][k];
            int d0 = T.body_dof0[a];
            for (int c = 0; c < 3; ++c) {
                float uu = L.u0[d0 + c];
                for (int x = 0; x < 6; ++x) V[x] += L.S[d0 + c][x] * uu;
            }
        }
        for (int x = 0; x < 6; ++x) L.V[lane][x] = V[x];
    }
    sync();
}

// ---------------------------------------------------------------------------------- one substep
HE_DEV void substep(Lds& L, float* Z, float* A, int mpad, const PhysArgs& a, const he_model& m, const PhysTopo& T,
                    int lane, const float* mass_scale, float mu, int tkind, unsigned long long* stamps,
                    unsigned long long& t_prev) {
    const he_sim_params& p = a.p;
    const float dt = p.dt;
    kinematics(L, m, T, lane);
    STAMP(0);
    const f3 o = f3{L.root_pos[0], L.root_pos[1], L.root_pos[2]};
    // ---- body spatial inertias about o
    if (lane < NB) {
        int b = lane;
        float ms = mass_scale ? mass_scale[b] : 1.f;
        float mass = m.mass[b] * ms;
        f4 q = f4{L.qw[b][0], L.qw[b][1], L.qw[b][2], L.qw[b][3]};
        f3 c0, c1, c2;
        qcols(q, c0, c1, c2);
        f3 cw = qapply(q, f3{m.com[b][0], m.com[b][1], m.com[b][2]});
        f3 s = f3{L.pw[b][0], L.pw[b][1], L.pw[b][2]} + cw - o;
        const float* in = m.inertia[b];
        // R Ib R^T: columns of R are c0 c1 c2 ; Ib symmetric
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
        float* o10 = L.Ib[b];
        o10[0] = mass; o10[1] = mass * s.x; o10[2] = mass * s.y; o10[3] = mass * s.z;
        o10[4] = I[0][0]; o10[5] = I[1][1]; o10[6] = I[2][2]; o10[7] = I[0][1]; o10[8] = I[0][2]; o10[9] = I[1][2];
        // ---- RNEA bias acceleration along the chain
        float Acc[6];
        f3 vxw = cross3(f3{L.u0[3], L.u0[4], L.u0[5]}, f3{L.u0[0], L.u0[1], L.u0[2]});
        Acc[0] = 0.f; Acc[1] = 0.f; Acc[2] = 0.f;
        Acc[3] = vxw.x - p.gravity[0]; Acc[4] = vxw.y - p.gravity[1]; Acc[5] = vxw.z - p.gravity[2];
        int depth = T.body_depth[b];
        for (int k = 1; k <= depth; ++k) {
            int ab = T.body_chain[b][k];
            int d0 = T.body_dof0[ab];
            for (int c = 0; c < 3; ++c) {
                float cr[6];
                crm(L.V[ab], L.S[d0 + c], cr);
                float uu = L.u0[d0 + c];
                for (int x = 0; x < 6; ++x) Acc[x] += cr[x] * uu;
            }
        }
        float IA[6], IV[6], X[6];
        si_apply(o10, Acc, IA);
        si_apply(o10, L.V[b], IV);
        crf(L.V[b], IV, X);
        for (int x = 0; x < 6; ++x) L.Acc[b][x] = IA[x] + X[x];  // body force f_b
    }
    sync();
    STAMP(1);
    // ---- subtree sums: F_b (forces) and composite inertias
    if (lane < NB) {
        uint32_t sm = T.sub_mask[lane];
        float Fs[6] = {0, 0, 0, 0, 0, 0}, Ics[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int d = 0; d < NB; ++d)
            if (sm >> d & 1u) {
                for (int x = 0; x < 6; ++x) Fs[x] += L.Acc[d][x];
                for (int x = 0; x < 10; ++x) Ics[x] += L.Ib[d][x];
            }
        for (int x = 0; x < 6; ++x) L.F[lane][x] = Fs[x];
        for (int x = 0; x < 10; ++x) L.Ic[lane][x] = Ics[x];
    }
    sync();
    STAMP(2);
    // ---- bias forces, IS_i = Ic S_i, drives
    for (int i = lane; i < NG; i += W) {
        int b = T.dof_body[i];
        float bias = dot6(L.S[i], L.F[b]);
        si_apply(L.Ic[b], L.S[i], L.IS[i]);
        float rhs = -bias, cf = 0.f;
        if (i >= 6) {
            int d = i - 6;
            float kp = m.stiffness[d] * p.kp_scale, kd = m.damping[d] * p.kd_scale;
            float err = L.tgt[d] - L.q[d];
            float u = L.u0[i];
            float tau = kp * (err - dt * u) - kd * u;
            float lim = m.effort[d];
            if (fabsf(tau) > lim) { tau = tau > 0.f ? lim : -lim; kp = 0.f; kd = 0.f; }
            L.dforce[d] = tau;
            rhs += tau;
            cf = dt * kp + kd;
        }
        L.rhs[i] = dt * rhs;
        L.coef[i] = cf;
    }
    sync();
    STAMP(3);
    // ---- CRBA entries H(i, j) = S_j . IS_i for j in chain(i); + armature + implicit drive terms
    for (int e = lane; e < T.nnz; e += W) {
        int i = T.ent_row[e], pos = e - T.row_start[i];
        int j = T.dof_chain[i][pos];
        float h = dot6(L.S[j], L.IS[i]);
        if (j == i && i >= 6) h += m.armature[i - 6] + dt * L.coef[i];
        L.H[e] = h;
    }
    sync();
    STAMP(4);
    // ---- sparse LTDL (RBDA 6.5) by dof level: all dofs with the same chain length are eliminated
    // together (their updates only touch shared ancestors -> LDS float atomics); rows are scaled
    // by their pivots in one pass at the end.
    for (int len = T.num_levels; len >= 2; --len) {
        const int d = len - 1, npairs = d * (d + 1) / 2;
        const int k0 = T.level_start[len - 1], total = (T.level_start[len] - k0) * npairs;
        for (int t = lane; t < total; t += W) {
            int kk = t / npairs, pr = t - kk * npairs;
            int k = T.level_dofs[k0 + kk];
            int rk = T.row_start[k];
            int ix = T.tri_i[pr], jx = T.tri_j[pr];
            int i = T.dof_chain[k][ix];
            atomicAdd(&L.H[T.row_start[i] + jx], -L.H[rk + ix] * L.H[rk + jx] / L.H[rk + d]);
        }
        sync();
    }
    for (int i = lane; i < NG; i += W) L.Dinv[i] = 1.0f / L.H[T.row_start[i] + T.dof_nanc[i] - 1];
    sync();
    for (int e = lane; e < T.nnz; e += W) {
        int i = T.ent_row[e];
        if (e - T.row_start[i] < T.dof_nanc[i] - 1) L.H[e] *= L.Dinv[i];
    }
    for (int i = lane; i < NG; i += W) L.y[i] = L.rhs[i];
    sync();
    STAMP(5);
    // ---- free velocity: du = L^-1 D^-1 L^-T rhs (both sweeps level-parallel)
    for (int len = T.num_levels; len >= 2; --len) {  // L^-T: push to ancestors, deepest level first
        const int d = len - 1, k0 = T.level_start[len - 1], total = (T.level_start[len] - k0) * d;
        for (int t = lane; t < total; t += W) {
            int kk = t / d, x = t - kk * d;
            int k = T.level_dofs[k0 + kk];
            atomicAdd(&L.y[T.dof_chain[k][x]], -L.H[T.row_start[k] + x] * L.y[k]);
        }
        sync();
    }
    for (int i = lane; i < NG; i += W) L.y[i] *= L.Dinv[i];
    sync();
    for (int lv = 1; lv < T.num_levels; ++lv) {  // L^-1: pull from ancestors, shallowest first
        for (int t = T.level_start[lv] + lane; t < T.level_start[lv + 1]; t += W) {
            int k = T.level_dofs[t];
            int rk = T.row_start[k];
            float acc = L.y[k];
            for (int x = 0; x < lv; ++x) acc -= L.H[rk + x] * L.y[T.dof_chain[k][x]];
            L.y[k] = acc;
        }
        sync();
        STAMP(6);
    }
    for (int i = lane; i < NG; i += W) L.uf[i] = L.u0[i] + L.y[i];
    // ---- contacts: terrain (bodies in order, box corners deepest-first), then self pairs
    const int maxc = p.max_contacts < MAXC ? p.max_contacts : MAXC;
    const float off = p.contact_offset;
    int nc = 0;
    {
        // per body: sphere 1, capsule 2 (end spheres), box up to 4 deepest corners (ranked by depth,
        // ties by corner index -- the oracle's selection order); fully unrolled, no scratch arrays
        int b = lane < NB ? lane : 0;
        const float* g = m.geom_params[b];
        int gt = m.geom_type[b];
        float cd[8];
        f3 cxs[8], cns[8];
        bool cand[8];
#pragma unroll
        for (int ci = 0; ci < 8; ++ci) { cand[ci] = false; cd[ci] = 0.f; }
        if (lane < NB) {
            if (gt == HE_GEOM_SPHERE) {
                f3 c = body_point(L, b, f3{g[0], g[1], g[2]});
                cd[0] = terrain_dist(p, tkind, c, cns[0]) - g[3];
                cxs[0] = c - cns[0] * g[3];
                cand[0] = cd[0] < off;
            } else if (gt == HE_GEOM_CAPSULE) {
#pragma unroll
                for (int e2 = 0; e2 < 2; ++e2) {
                    f3 c = body_point(L, b, f3{g[3 * e2], g[3 * e2 + 1], g[3 * e2 + 2]});
                    cd[e2] = terrain_dist(p, tkind, c, cns[e2]) - g[6];
                    cxs[e2] = c - cns[e2] * g[6];
                    cand[e2] = cd[e2] < off;
                }
            } else {
                f4 bq = f4{g[6], g[7], g[8], g[9]};
#pragma unroll
                for (int ci = 0; ci < 8; ++ci) {
                    f3 lb = f3{(ci & 1) ? g[3] : -g[3], (ci & 2) ? g[4] : -g[4], (ci & 4) ? g[5] : -g[5]};
                    cxs[ci] = body_point(L, b, f3{g[0], g[1], g[2]} + qapply(bq, lb));
                    cd[ci] = terrain_dist(p, tkind, cxs[ci], cns[ci]);
                    cand[ci] = cd[ci] < off;
                }
            }
        }
        int rank[8];
        int myn = 0;
#pragma unroll
        for (int ci = 0; ci < 8; ++ci) {
            int rk = 0;
#pragma unroll
            for (int cj = 0; cj < 8; ++cj) {
                // box corners by depth; sphere / capsule end points in geometric order
                bool before = gt == HE_GEOM_BOX ? (cd[cj] < cd[ci] || (cd[cj] == cd[ci] && cj < ci)) : cj < ci;
                if (cand[cj] && before) ++rk;
            }
            rank[ci] = rk;
            if (cand[ci] && rk < 4) ++myn;
        }
        int incl = myn;
        for (int s2 = 1; s2 < W; s2 <<= 1) {
            int v = __shfl_up(incl, s2, W);
            if (lane >= s2) incl += v;
        }
        int total = __shfl(incl, W - 1, W);
        int base = incl - myn;
#pragma unroll
        for (int ci = 0; ci < 8; ++ci)
            if (cand[ci] && rank[ci] < 4 && base + rank[ci] < maxc)
                store_contact(L, base + rank[ci], b, -1, cxs[ci], cns[ci], cd[ci], mu);
        nc = total < maxc ? total : maxc;
    }
    if (p.self_collision && nc < maxc) {
        for (int base = 0; base < m.num_pairs; base += W) {
            int pi = base + lane;
            bool hit = false;
            f3 x, n;
            float gap = 0.f;
            int i = 0, j = 0;
            if (pi < m.num_pairs) {
                i = m.pairs[pi][0];
                j = m.pairs[pi][1];
                f3 a0, a1, b0, b1, ci, cj;
                float ri, rj;
                body_segment(m, L, i, a0, a1, ri);
                body_segment(m, L, j, b0, b1, rj);
                seg_seg(a0, a1, b0, b1, ci, cj);
                f3 dv = ci - cj;
                float len = norm3(dv);
                gap = len - ri - rj;
                if (gap < off) {
                    hit = true;
                    n = len > 1e-9f ? dv * (1.0f / len) : f3{0.f, 0.f, 1.f};
                    x = cj + n * (rj + 0.5f * gap);
                }
            }
            int total;
            int pre = wave_prefix(hit, lane, total);
            if (hit && nc + pre < maxc) store_contact(L, nc + pre, i, j, x, n, gap, mu);
            nc = nc + total < maxc ? nc + total : maxc;
        }
    }
    if (lane == 0) L.nc = nc;
    if (lane < NB) { L.cf[lane][0] = 0.f; L.cf[lane][1] = 0.f; L.cf[lane][2] = 0.f; }
    sync();
    STAMP(7);
    if (nc > 0) {
        const int nr = 3 * nc;
        // ---- contact rows: Z[i][r] = J_r^T (dense over the 75 dofs), brow = J_r uf + bias
        for (int t = lane; t < NG * nr; t += W) {
            int i = t / nr, r = t - i * nr;
            int ci = r / 3, kind = r - 3 * ci;
            const float* dir = kind == 0 ? L.cn[ci] : (kind == 1 ? L.ct1[ci] : L.ct2[ci]);
            int bi = T.dof_body[i];
            float sgn = (T.anc_mask[L.cb0[ci]] >> bi & 1u) ? 1.f : 0.f;
            if (L.cb1[ci] >= 0 && (T.anc_mask[L.cb1[ci]] >> bi & 1u)) sgn -= 1.f;
            float z = 0.f;
            if (sgn != 0.f) {
                f3 xo = f3{L.cx[ci][0], L.cx[ci][1], L.cx[ci][2]} - o;
                f3 dd = f3{dir[0], dir[1], dir[2]};
                f3 rho = cross3(xo, dd);
                const float* S = L.S[i];
                z = sgn * (S[0] * rho.x + S[1] * rho.y + S[2] * rho.z + S[3] * dd.x + S[4] * dd.y + S[5] * dd.z);
            }
            Z[i * mpad + r] = z;
        }
        sync();
        for (int r = lane; r < nr; r += W) {
            float ju = 0.f;
            for (int i = 0; i < NG; ++i) ju += Z[i * mpad + r] * L.uf[i];
            int ci = r / 3;
            float bb = 0.f;
            if (r - 3 * ci == 0) {
                float g = L.cgap[ci];
                bb = g >= 0.f ? g / dt : fmaxf(p.baumgarte * g / dt, -p.max_depenetration_velocity);
            }
            L.brow[r] = ju + bb;
            // Z <- L^-T Z for row r (owned by this lane); a terrain row is supported on one chain
            if (L.cb1[ci] < 0) {
                const int8_t* ch = T.dof_chain[T.body_last_dof[L.cb0[ci]]];
                int len = T.dof_nanc[T.body_last_dof[L.cb0[ci]]];
                for (int x = len - 1; x > 0; --x) {
                    int k = ch[x];
                    float zk = Z[k * mpad + r];
                    int rk = T.row_start[k];
                    for (int y = 0; y < x; ++y) Z[ch[y] * mpad + r] -= L.H[rk + y] * zk;
                }
            } else {
                for (int k = NG - 1; k > 0; --k) {
                    float zk = Z[k * mpad + r];
                    if (zk == 0.f) continue;
                    int d = T.dof_nanc[k] - 1;
                    int rk = T.row_start[k];
                    for (int x = 0; x < d; ++x) Z[T.dof_chain[k][x] * mpad + r] -= L.H[rk + x] * zk;
                }
            }
        }
        sync();
        STAMP(8);
        // ---- Delassus A = Z^T D^-1 Z (full symmetric, row r contiguous), summed over the
        // support chain of whichever row is a terrain row
        for (int t = lane; t < nr * nr; t += W) {
            int r = t / nr, c = t - r * nr;
            if (c > r) continue;
            int cr = r / 3, cc = c / 3;
            float acc = 0.f;
            int b = L.cb1[cr] < 0 ? L.cb0[cr] : (L.cb1[cc] < 0 ? L.cb0[cc] : -1);
            if (b >= 0) {
                int ld = T.body_last_dof[b];
                const int8_t* ch = T.dof_chain[ld];
                int len = T.dof_nanc[ld];
                for (int x = 0; x < len; ++x) {
                    int i = ch[x];
                    acc += Z[i * mpad + r] * Z[i * mpad + c] * L.Dinv[i];
                }
            } else {
                for (int i = 0; i < NG; ++i) acc += Z[i * mpad + r] * Z[i * mpad + c] * L.Dinv[i];
            }
            A[r * mpad + c] = acc;
            A[c * mpad + r] = acc;
        }
        sync();
        STAMP(9);
        // ---- projected Gauss-Seidel; lane l keeps residual w and impulse for rows l and l+64
        float w0 = lane < nr ? L.brow[lane] : 0.f, w1 = lane + W < nr ? L.brow[lane + W] : 0.f;
        float l0 = 0.f, l1 = 0.f;
        for (int it = 0; it < p.solver_iterations; ++it) {
            for (int ci = 0; ci < nc; ++ci) {
                float lamn = 0.f;
                for (int kind = 0; kind < 3; ++kind) {
                    int r = 3 * ci + kind;
                    float wr = r < W ? __shfl(w0, r, W) : __shfl(w1, r - W, W);
                    float lr = r < W ? __shfl(l0, r, W) : __shfl(l1, r - W, W);
                    float arr = A[r * mpad + r] + 1e-12f;
                    float nl = lr - wr / arr;
                    if (kind == 0) { nl = fmaxf(nl, 0.f); lamn = nl; }
                    else { float bnd = L.cmu[ci] * lamn; nl = fminf(fmaxf(nl, -bnd), bnd); }
                    float del = nl - lr;
                    if (del != 0.f) {
                        if (lane < nr) w0 += A[r * mpad + lane] * del;
                        if (lane + W < nr) w1 += A[r * mpad + lane + W] * del;
                        if (r < W) { if (lane == r) l0 = nl; } else { if (lane == r - W) l1 = nl; }
                    }
                }
            }
        }
        // ---- du = L^-1 D^-1 (Z lambda)
        if (lane < nr) L.brow[lane] = l0;
        if (lane + W < nr) L.brow[lane + W] = l1;
        sync();
        STAMP(10);
        for (int i = lane; i < NG; i += W) {
            float acc = 0.f;
            for (int r = 0; r < nr; ++r) acc += Z[i * mpad + r] * L.brow[r];
            L.y[i] = acc * L.Dinv[i];
        }
        sync();
        for (int lv = 1; lv < T.num_levels; ++lv) {
            for (int t = T.level_start[lv] + lane; t < T.level_start[lv + 1]; t += W) {
                int k = T.level_dofs[t];
                int rk = T.row_start[k];
                float acc = L.y[k];
                for (int x = 0; x < lv; ++x) acc -= L.H[rk + x] * L.y[T.dof_chain[k][x]];
                L.y[k] = acc;
            }
            sync();
        }
        for (int i = lane; i < NG; i += W) L.uf[i] += L.y[i];
        if (lane < NB) {
            float fx = 0.f, fy = 0.f, fz = 0.f;
            for (int ci = 0; ci < nc; ++ci) {
                float s = L.cb0[ci] == lane ? 1.f : (L.cb1[ci] == lane ? -1.f : 0.f);
                if (s == 0.f) continue;
                float ln = L.brow[3 * ci], la = L.brow[3 * ci + 1], lb = L.brow[3 * ci + 2];
                fx += s * (ln * L.cn[ci][0] + la * L.ct1[ci][0] + lb * L.ct2[ci][0]);
                fy += s * (ln * L.cn[ci][1] + la * L.ct1[ci][1] + lb * L.ct2[ci][1]);
                fz += s * (ln * L.cn[ci][2] + la * L.ct1[ci][2] + lb * L.ct2[ci][2]);
            }
            L.cf[lane][0] = fx / dt; L.cf[lane][1] = fy / dt; L.cf[lane][2] = fz / dt;
        }
        sync();
        STAMP(11);
    }
    // ---- drive force actually applied, damping, clamps, write velocities
    const float damp = 1.0f / (1.0f + dt * p.angular_damping);
    for (int i = lane; i < NG; i += W) {
        if (i >= 6) L.dforce[i - 6] -= L.coef[i] * (L.uf[i] - L.u0[i]);
    }
    sync();
    if (lane < NB) {
        int d0 = lane == 0 ? 0 : 6 + 3 * (lane - 1);
        float w[3] = {L.uf[d0] * damp, L.uf[d0 + 1] * damp, L.uf[d0 + 2] * damp};
        float nrm = sqrtf(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
        if (nrm > p.max_angular_velocity) {
            float s = p.max_angular_velocity / nrm;
            w[0] *= s; w[1] *= s; w[2] *= s;
        }
        L.u0[d0] = w[0]; L.u0[d0 + 1] = w[1]; L.u0[d0 + 2] = w[2];
        if (lane == 0) { L.u0[3] = L.uf[3]; L.u0[4] = L.uf[4]; L.u0[5] = L.uf[5]; }
    }
    sync();
    // ---- semi-implicit position update
    if (lane < NB) {
        if (lane == 0) {
            for (int c = 0; c < 3; ++c) L.root_pos[c] += dt * L.u0[3 + c];
            f4 dq = qexp(f3{dt * L.u0[0], dt * L.u0[1], dt * L.u0[2]});
            f4 nq = qnormalize(qmul(dq, f4{L.root_q[0], L.root_q[1], L.root_q[2], L.root_q[3]}));
            L.root_q[0] = nq.x; L.root_q[1] = nq.y; L.root_q[2] = nq.z; L.root_q[3] = nq.w;
        } else {
            int d = 3 * (lane - 1), g = 6 + d;
            f4 ql = qexp(f3{L.q[d], L.q[d + 1], L.q[d + 2]});
            f4 dq = qexp(f3{dt * L.u0[g], dt * L.u0[g + 1], dt * L.u0[g + 2]});
            f3 nv = qlog(qnormalize(qmul(ql, dq)));
            L.q[d] = nv.x; L.q[d + 1] = nv.y; L.q[d + 2] = nv.z;
        }
    }
    sync();
    STAMP(12);
}

__global__ void __launch_bounds__(64) physics_kernel(PhysArgs a, int mpad) {
    extern __shared__ float smem[];
    Lds& L = *reinterpret_cast<Lds*>(smem);
    float* Z = smem + (sizeof(Lds) + 3) / 4;
    float* A = Z + NG * mpad;
    const int e = blockIdx.x;
    const int lane = threadIdx.x;
    const he_model& m = *a.model;
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.topo);
        uint32_t* dst = reinterpret_cast<uint32_t*>(&L.T);
        for (int i = lane; i < (int)(sizeof(PhysTopo) / 4); i += W) dst[i] = src[i];
    }
    const PhysTopo& T = L.T;
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
    sync();
    const float* ms = a.mass_scale ? a.mass_scale + (size_t)e * NB : nullptr;
    float mu = a.friction ? a.friction[e] : a.p.friction;
    int tk = (a.p.terrain && a.terrain_kind) ? a.terrain_kind[e] : 0;
    unsigned long long* stamps = a.stamps ? a.stamps + (size_t)e * 16 : nullptr;
    unsigned long long t_prev = __builtin_readcyclecounter();
    for (int s = 0; s < a.substeps; ++s) substep(L, Z, A, mpad, a, m, T, lane, ms, mu, tk, stamps, t_prev);
    // ---- outputs: generalized state, FK rigid-body state, forces
    kinematics(L, m, T, lane);
    STAMP(13);
    float* rso = a.root_states + (size_t)e * 13;
    if (lane < 3) { rso[lane] = L.root_pos[lane]; rso[7 + lane] = L.u0[3 + lane]; rso[10 + lane] = L.u0[lane]; }
    if (lane < 4) rso[3 + lane] = L.root_q[lane];
    for (int d = lane; d < ND; d += W) {
        a.dof_state[((size_t)e * ND + d) * 2] = L.q[d];
        a.dof_state[((size_t)e * ND + d) * 2 + 1] = L.u0[6 + d];
        a.dof_force[(size_t)e * ND + d] = L.dforce[d];
    }
    for (int t = lane; t < NB * 13; t += W) {
        int b = t / 13, c = t - 13 * b;
        float v;
        if (c < 3) v = L.pw[b][c];
        else if (c < 7) v = L.qw[b][c - 3];
        else if (c < 10) {
            f3 w = f3{L.V[b][0], L.V[b][1], L.V[b][2]};
            f3 r = f3{L.pw[b][0] - L.root_pos[0], L.pw[b][1] - L.root_pos[1], L.pw[b][2] - L.root_pos[2]};
            f3 vv = f3{L.V[b][3], L.V[b][4], L.V[b][5]} + cross3(w, r);
            v = c == 7 ? vv.x : (c == 8 ? vv.y : vv.z);
        } else v = L.V[b][c - 10];
        a.rb_state[(size_t)e * NB * 13 + t] = v;
    }
    for (int t = lane; t < NB * 3; t += W) a.contact_forces[(size_t)e * NB * 3 + t] = L.cf[t / 3][t % 3];
    if (lane == 0 && a.num_contacts) a.num_contacts[e] = L.nc;
}

}  // namespace

size_t physics_lds_bytes(int max_contacts, int* mpad_out) {
    int m = 3 * (max_contacts < 1 ? 1 : (max_contacts > MAXC ? MAXC : max_contacts));
    int mpad = m;
    if (mpad_out) *mpad_out = mpad;
    return ((sizeof(Lds) + 3) / 4) * 4 + (size_t)(NG * mpad + mpad * mpad) * sizeof(float);
}

hipError_t launch_physics(const PhysArgs& a, hipStream_t stream) {
    if (a.num_envs <= 0) return hipSuccess;
    int mpad = 0;
    size_t lds = physics_lds_bytes(a.p.max_contacts, &mpad);
    hipError_t err = hipFuncSetAttribute(reinterpret_cast<const void*>(physics_kernel),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (err != hipSuccess) return err;
    physics_kernel<<<a.num_envs, W, lds, stream>>>(a, mpad);
    return hipGetLastError();
}
