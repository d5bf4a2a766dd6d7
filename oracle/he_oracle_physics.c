/*
 * he_oracle_physics.c -- TEST INFRASTRUCTURE ONLY (see he_oracle.c header).
 *
 * Scalar fp64 reference of the engine's articulated-body step. It replaces
 * gym.simulate (puffer_phc/envs/humanoid_phc.py:131-134) whose PhysX implementation is closed
 * and absent: PHYSICS PARITY VS ISAAC GYM IS UNPINNED. Constants follow
 * puffer_phc/envs/isaacgym_env.py:6-35 (dt 1/60, gravity, contact offset 0.02, max depenetration
 * 10), asset options humanoid_phc.py:211-214 (angular damping 0.01, max angular velocity 100),
 * PD drives humanoid_phc.py:276-280 and the self-collision filter humanoid_phc.py:370-381.
 *
 * Algorithm per substep (generalized velocity u = [w_root(3), v_root(3), joint(69)],
 * joint velocity = relative angular velocity in the child frame, joint position = exp map):
 *   FK -> spatial axes S about the root origin o -> RNEA bias (gravity + Coriolis)
 *   -> CRBA mass matrix + armature -> implicit PD (effort limit: the drive scaled down)
 *   -> branch-induced sparse LTDL factorisation -> free velocity
 *   -> ground + self contacts (speculative within contact_offset) -> Delassus A = Z^T D^-1 Z
 *      with Z = L^-T J^T -> projected Gauss-Seidel (pyramidal friction) -> velocity update
 *   -> damping / clamps -> semi-implicit position update.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../include/humanoid_engine.h"

typedef double R;
#define NB HE_NUM_BODIES
#define ND HE_NUM_DOF
#define NG HE_NUM_GEN
/* The oracle's own capacity: max_contacts above the engine's HE_MAX_CONTACTS lifts the slot and
 * row caps (HE_MAX_ROWS) so that the engine's truncation becomes visible
 * (tests/diag/truncation_effect.py); the warm-start cache holds HE_MAX_ROWS rows. */
#define MAXC 64
#define MAXROW (3 * MAXC)

/* Sensitivity probes (tests/test_gpu_parity.py _cond_close): rounding-level noise on the Delassus
 * operator and the contact right-hand side, A_rc (1 + rel xi), b_r (1 + rel xi) with xi uniform in
 * [-1, 1] hashed from (seed, env, physics step, r, c). A resting body's contacts are statically
 * indeterminate (A nearly singular), and how the impulses spread over them -- which friction row
 * reaches its bound first -- moves with A's rounding as much as with the state's: the fp32 engine
 * rounds A in every step. 0 (the default) = off. Test infrastructure only. */
static double g_probe_rel = 0.0;
static uint64_t g_probe_seed = 0;
static __thread int g_probe_env, g_probe_sub;
void ho_set_probe_noise(uint64_t seed, double rel) { g_probe_seed = seed; g_probe_rel = rel; }
/* diagnostic (tests/diag): friction bounds from the normal impulses at the sweep's start (1)
 * instead of the current ones (0, the engine's) */
static int g_lagged_bounds = 0;
void ho_set_lagged_bounds(int on) { g_lagged_bounds = on; }
static double probe_xi(int r, int c) {
    uint64_t z = g_probe_seed * 0x9E3779B97F4A7C15ull ^ ((uint64_t)g_probe_env + 0x632BE59BD9B4E019ull) * 0xBF58476D1CE4E5B9ull ^
                 ((uint64_t)g_probe_sub * 4099u + (uint64_t)r * 131u + (uint64_t)c + 0x2545F4914F6CDD1Dull) * 0x94D049BB133111EBull;
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

typedef struct topo {
    int dof_parent[NG];
    int dof_body[NG];
    int body_dof0[NB];
    int is_anc[NB][NB]; /* is_anc[a][b]: a is ancestor-or-self of b */
} topo;

static void build_topo(const he_model* m, topo* t) {
    for (int i = 0; i < 6; ++i) { t->dof_parent[i] = i - 1; t->dof_body[i] = 0; }
    t->body_dof0[0] = 0;
    for (int b = 1; b < NB; ++b) {
        int d0 = 6 + 3 * (b - 1);
        t->body_dof0[b] = d0;
        int p = m->parents[b];
        int plast = p == 0 ? 5 : 6 + 3 * (p - 1) + 2;
        for (int c = 0; c < 3; ++c) {
            t->dof_parent[d0 + c] = c == 0 ? plast : d0 + c - 1;
            t->dof_body[d0 + c] = b;
        }
    }
    memset(t->is_anc, 0, sizeof(t->is_anc));
    for (int b = 0; b < NB; ++b)
        for (int a = b; a >= 0; a = m->parents[a]) { t->is_anc[a][b] = 1; if (a == 0) break; }
}

/* ---------------------------------------------------------------- small math */
static inline R dot3(const R* a, const R* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void cross3(const R* a, const R* b, R* o) {
    R x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}
static void qmul(const R* a, const R* b, R* o) { /* Hamilton, xyzw */
    R x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    R y = a[3] * b[1] - a[0] * b[2] + a[1] * b[3] + a[2] * b[0];
    R z = a[3] * b[2] + a[0] * b[1] - a[1] * b[0] + a[2] * b[3];
    R w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    o[0] = x; o[1] = y; o[2] = z; o[3] = w;
}
static void qnormalize(R* q) {
    R n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (n < 1e-12) { q[0] = q[1] = q[2] = 0; q[3] = 1; return; }
    for (int i = 0; i < 4; ++i) q[i] /= n;
}
static void qexp(const R* v, R* q) { /* rotation vector -> unit quaternion */
    R th = sqrt(dot3(v, v));
    if (th < 1e-8) { q[0] = 0.5 * v[0]; q[1] = 0.5 * v[1]; q[2] = 0.5 * v[2]; q[3] = 1; qnormalize(q); return; }
    R s = sin(0.5 * th) / th;
    q[0] = v[0] * s; q[1] = v[1] * s; q[2] = v[2] * s; q[3] = cos(0.5 * th);
}
static void qlog(const R* qin, R* v) { /* minimal rotation vector, |angle| <= pi */
    R q[4] = {qin[0], qin[1], qin[2], qin[3]};
    if (q[3] < 0) for (int i = 0; i < 4; ++i) q[i] = -q[i];
    R s = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
    if (s < 1e-8) { v[0] = 2 * q[0]; v[1] = 2 * q[1]; v[2] = 2 * q[2]; return; }
    R th = 2 * atan2(s, q[3]);
    v[0] = q[0] / s * th; v[1] = q[1] / s * th; v[2] = q[2] / s * th;
}
static void qmat(const R* q, R m[3][3]) {
    R x = q[0], y = q[1], z = q[2], w = q[3];
    m[0][0] = 1 - 2 * (y * y + z * z); m[0][1] = 2 * (x * y - z * w); m[0][2] = 2 * (x * z + y * w);
    m[1][0] = 2 * (x * y + z * w); m[1][1] = 1 - 2 * (x * x + z * z); m[1][2] = 2 * (y * z - x * w);
    m[2][0] = 2 * (x * z - y * w); m[2][1] = 2 * (y * z + x * w); m[2][2] = 1 - 2 * (x * x + y * y);
}
static inline void matvec(R m[3][3], const R* v, R* o) {
    R a = m[0][0] * v[0] + m[0][1] * v[1] + m[0][2] * v[2];
    R b = m[1][0] * v[0] + m[1][1] * v[1] + m[1][2] * v[2];
    R c = m[2][0] * v[0] + m[2][1] * v[1] + m[2][2] * v[2];
    o[0] = a; o[1] = b; o[2] = c;
}

/* spatial inertia about o: (m, h = m*(c-o), I3 about o) ; f = I V with V = (w, v):
 *   n = I3 w + h x v ;  f = m v - h x w */
typedef struct sinertia { R m, h[3], I[3][3]; } sinertia;
static void si_apply(const sinertia* I, const R* V, R* F) {
    R hv[3], hw[3];
    cross3(I->h, V + 3, hv);
    cross3(I->h, V, hw);
    for (int r = 0; r < 3; ++r) {
        F[r] = I->I[r][0] * V[0] + I->I[r][1] * V[1] + I->I[r][2] * V[2] + hv[r];
        F[3 + r] = I->m * V[3 + r] - hw[r];
    }
}
static void si_add(sinertia* a, const sinertia* b) {
    a->m += b->m;
    for (int r = 0; r < 3; ++r) { a->h[r] += b->h[r]; for (int c = 0; c < 3; ++c) a->I[r][c] += b->I[r][c]; }
}
/* motion cross: V x W */
static void crm(const R* V, const R* W, R* O) {
    R a[3], b[3], c[3];
    cross3(V, W, a);
    cross3(V, W + 3, b);
    cross3(V + 3, W, c);
    for (int i = 0; i < 3; ++i) { O[i] = a[i]; O[3 + i] = b[i] + c[i]; }
}
/* force cross: V x* F */
static void crf(const R* V, const R* F, R* O) {
    R a[3], b[3], c[3];
    cross3(V, F, a);
    cross3(V + 3, F + 3, b);
    cross3(V, F + 3, c);
    for (int i = 0; i < 3; ++i) { O[i] = a[i] + b[i]; O[3 + i] = c[i]; }
}

/* ---------------------------------------------------------------- env state */
typedef struct env_state {
    R root_pos[3], root_q[4], root_v[3], root_w[3];
    R q[ND], u[ND], target[ND];
} env_state;

typedef struct kin {
    R qw[NB][4];     /* body world rotation */
    R Rw[NB][3][3];
    R pw[NB][3];     /* body origin */
    R o[3];
    R S[NG][6];
    R V[NB][6];
} kin;

static void kinematics(const he_model* m, const topo* t, const env_state* s, kin* k) {
    memcpy(k->qw[0], s->root_q, sizeof(R) * 4);
    qnormalize(k->qw[0]);
    memcpy(k->pw[0], s->root_pos, sizeof(R) * 3);
    qmat(k->qw[0], k->Rw[0]);
    for (int b = 1; b < NB; ++b) {
        int p = m->parents[b];
        R ql[4], lp[3] = {m->local_pos[b][0], m->local_pos[b][1], m->local_pos[b][2]}, off[3];
        qexp(&s->q[3 * (b - 1)], ql);
        qmul(k->qw[p], ql, k->qw[b]);
        qmat(k->qw[b], k->Rw[b]);
        matvec(k->Rw[p], lp, off);
        for (int c = 0; c < 3; ++c) k->pw[b][c] = k->pw[p][c] + off[c];
    }
    memcpy(k->o, k->pw[0], sizeof(R) * 3);
    memset(k->S, 0, sizeof(k->S));
    for (int c = 0; c < 3; ++c) { k->S[c][c] = 1; k->S[3 + c][3 + c] = 1; }
    for (int b = 1; b < NB; ++b) {
        R r[3] = {k->pw[b][0] - k->o[0], k->pw[b][1] - k->o[1], k->pw[b][2] - k->o[2]};
        for (int c = 0; c < 3; ++c) {
            R a[3] = {k->Rw[b][0][c], k->Rw[b][1][c], k->Rw[b][2][c]}, l[3];
            cross3(r, a, l);
            R* S = k->S[t->body_dof0[b] + c];
            S[0] = a[0]; S[1] = a[1]; S[2] = a[2]; S[3] = l[0]; S[4] = l[1]; S[5] = l[2];
        }
    }
    /* body spatial velocities about o */
    k->V[0][0] = s->root_w[0]; k->V[0][1] = s->root_w[1]; k->V[0][2] = s->root_w[2];
    k->V[0][3] = s->root_v[0]; k->V[0][4] = s->root_v[1]; k->V[0][5] = s->root_v[2];
    for (int b = 1; b < NB; ++b) {
        int p = m->parents[b];
        for (int i = 0; i < 6; ++i) k->V[b][i] = k->V[p][i];
        for (int c = 0; c < 3; ++c) {
            R uu = s->u[3 * (b - 1) + c];
            for (int i = 0; i < 6; ++i) k->V[b][i] += k->S[t->body_dof0[b] + c][i] * uu;
        }
    }
}

static void body_inertia(const he_model* m, const kin* k, int b, R mass_scale, sinertia* I) {
    R mass = m->mass[b] * mass_scale;
    R com[3] = {m->com[b][0], m->com[b][1], m->com[b][2]}, cw[3];
    matvec((R(*)[3])k->Rw[b], com, cw);
    R s[3] = {k->pw[b][0] + cw[0] - k->o[0], k->pw[b][1] + cw[1] - k->o[1], k->pw[b][2] + cw[2] - k->o[2]};
    const float* in = m->inertia[b];
    R Ib[3][3] = {{in[0], in[3], in[4]}, {in[3], in[1], in[5]}, {in[4], in[5], in[2]}};
    R tmp[3][3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            R acc = 0;
            for (int x = 0; x < 3; ++x) acc += k->Rw[b][r][x] * Ib[x][c];
            tmp[r][c] = acc;
        }
    R ss = dot3(s, s);
    I->m = mass;
    for (int r = 0; r < 3; ++r) {
        I->h[r] = mass * s[r];
        for (int c = 0; c < 3; ++c) {
            R acc = 0;
            for (int x = 0; x < 3; ++x) acc += tmp[r][x] * k->Rw[b][c][x];
            I->I[r][c] = acc * mass_scale + mass * ((r == c ? ss : 0) - s[r] * s[c]);
        }
    }
}

/* ---------------------------------------------------------------- contacts */
/* A contact slot has three rows (normal, two friction directions). A joint-limit slot has the
 * limit row in the normal position and two zero rows (mu 0), so that limits and contacts share
 * one row layout and one Gauss-Seidel order with the engine. */
typedef struct contact {
    int b0, b1;       /* b1 = -1 for terrain, -2 for a joint limit (b0 = the joint's body) */
    int key;          /* warm-start key of its normal row: b0 | (b1 + 2) << 5 | sub << 10 */
    R x[3], n[3];
    R gap;
    R mu;
    R g[3];           /* joint limit: the row over the joint's three dofs */
} contact;

/* A solver row (patch friction; include/humanoid_engine.h HE_MAX_ROWS). Rows in Gauss-Seidel order:
 * for every slot its normal row (a joint limit: its one row); after the last point of a body's
 * terrain patch (the body's terrain slots, contiguous) the patch's friction rows: 2 tangential
 * rows at the points' centroid and, from 2 points on, 1 torsional row about the patch normal; a
 * self pair is a patch of its own point (2 tangential rows). PhysX runs patch friction (Isaac
 * Gym's default), with friction per body-ground patch rather than per point. */
typedef struct srow {
    int slot, kind;   /* kind 0 normal / limit, 1 and 2 tangential, 3 torsional */
    int n0, cnt;      /* friction rows: the patch's normal rows n0 .. n0 + cnt - 1 */
    int b0, b1;
    R dir[3], rho[3]; /* J = (rho, dir) about o: rho = (x - o) x dir; torsion rho = n_patch, dir = 0 */
    R muw;            /* friction bound |lambda| <= muw * (sum of the patch's normal impulses):
                         mu (tangential), mu r_patch (torsion: r_patch = the points' mean distance
                         from the centroid in the tangent plane) */
    int key;          /* 16-bit row key (include/humanoid_engine.h, the cache layout) */
} srow;

static R terrain_height(const he_sim_params* p, int kind, const R* x, R* n) {
    /* returns signed distance of x to the terrain surface along its normal n */
    if (kind == 1) {
        R s = sin(p->terrain_slope), c = cos(p->terrain_slope);
        n[0] = -s; n[1] = 0; n[2] = c;
        return dot3(n, x);
    }
    n[0] = 0; n[1] = 0; n[2] = 1;
    if (kind == 2) {
        R h = 0;
        if (x[0] > 0) h = p->step_height * floor(x[0] / p->step_length);
        return x[2] - h;
    }
    return x[2];
}

static void friction_basis(const R* n, R* t1, R* t2) {
    R a[3] = {1, 0, 0};
    if (fabs(n[0]) > 0.9) { a[0] = 0; a[1] = 1; }
    R d = dot3(a, n);
    for (int i = 0; i < 3; ++i) t1[i] = a[i] - d * n[i];
    R l = sqrt(dot3(t1, t1));
    for (int i = 0; i < 3; ++i) t1[i] /= l;
    cross3(n, t1, t2);
}

static void body_point(const kin* k, int b, const R* local, R* out) {
    R w[3];
    matvec((R(*)[3])k->Rw[b], local, w);
    for (int i = 0; i < 3; ++i) out[i] = k->pw[b][i] + w[i];
}

/* body collision proxy: segment (a, b) and radius */
static void body_segment(const he_model* m, const kin* k, int b, R* a, R* c, R* r) {
    const float* g = m->geom_params[b];
    if (m->geom_type[b] == HE_GEOM_SPHERE) {
        R l[3] = {g[0], g[1], g[2]};
        body_point(k, b, l, a);
        memcpy(c, a, sizeof(R) * 3);
        *r = g[3];
    } else if (m->geom_type[b] == HE_GEOM_CAPSULE) {
        R l0[3] = {g[0], g[1], g[2]}, l1[3] = {g[3], g[4], g[5]};
        body_point(k, b, l0, a);
        body_point(k, b, l1, c);
        *r = g[6];
    } else { /* box -> capsule proxy along its longest axis */
        R e[3] = {g[3], g[4], g[5]};
        int ax = 0;
        if (e[1] > e[ax]) ax = 1;
        if (e[2] > e[ax]) ax = 2;
        R rp = m->geom_radius[b];
        R half = e[ax] - rp;
        if (half < 0) half = 0;
        R bq[4] = {g[6], g[7], g[8], g[9]}, bm[3][3];
        qmat(bq, bm);
        R dir[3] = {bm[0][ax] * half, bm[1][ax] * half, bm[2][ax] * half};
        R l0[3] = {g[0] - dir[0], g[1] - dir[1], g[2] - dir[2]}, l1[3] = {g[0] + dir[0], g[1] + dir[1], g[2] + dir[2]};
        body_point(k, b, l0, a);
        body_point(k, b, l1, c);
        *r = rp;
    }
}

/* closest points between segments p1q1 and p2q2 (Ericson, RTCD 5.1.9) */
static void seg_seg(const R* p1, const R* q1, const R* p2, const R* q2, R* c1, R* c2) {
    R d1[3], d2[3], r[3];
    for (int i = 0; i < 3; ++i) { d1[i] = q1[i] - p1[i]; d2[i] = q2[i] - p2[i]; r[i] = p1[i] - p2[i]; }
    R a = dot3(d1, d1), e = dot3(d2, d2), f = dot3(d2, r);
    R s, t;
    const R eps = 1e-12;
    if (a <= eps && e <= eps) { s = t = 0; }
    else if (a <= eps) { s = 0; t = f / e; t = t < 0 ? 0 : (t > 1 ? 1 : t); }
    else {
        R c = dot3(d1, r);
        if (e <= eps) { t = 0; s = -c / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
        else {
            R b = dot3(d1, d2), den = a * e - b * b;
            s = den > eps ? (b * f - c * e) / den : 0;
            s = s < 0 ? 0 : (s > 1 ? 1 : s);
            t = (b * s + f) / e;
            if (t < 0) { t = 0; s = -c / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
            else if (t > 1) { t = 1; s = (b - c) / a; s = s < 0 ? 0 : (s > 1 ? 1 : s); }
        }
    }
    for (int i = 0; i < 3; ++i) { c1[i] = p1[i] + d1[i] * s; c2[i] = p2[i] + d2[i] * t; }
}

static int add_contact(contact* cs, int nc, int maxc, int* total, int b0, int b1, int sub, const R* x, const R* n,
                       R gap, R mu) {
    ++*total; /* every generated contact counts; the ones past the capacity are dropped */
    if (nc >= maxc) return nc;
    contact* c = &cs[nc];
    c->b0 = b0; c->b1 = b1;
    c->key = b0 | ((b1 + 2) << 5) | (sub << 10);
    memcpy(c->x, x, sizeof(R) * 3);
    memcpy(c->n, n, sizeof(R) * 3);
    c->gap = gap;
    c->mu = mu;
    c->g[0] = c->g[1] = c->g[2] = 0;
    return nc + 1;
}

/* Row c of the inverse right Jacobian of SO(3) at the rotation vector th: the rate of the
 * exp-map joint coordinates is J_r^-1(th) u for the joint's relative angular velocity u (child
 * frame), because the joint integrates exp(q+) = exp(q) exp(dt u).
 *   J_r^-1 = I + [th]x / 2 + k(|th|) [th]x^2,  k = 1/t^2 - cos(t/2) / (2 t sin(t/2)) */
static void jr_inv_row(const R* th, int c, R* row) {
    R t2 = dot3(th, th), t = sqrt(t2);
    R k = t < 1e-2 ? 1.0 / 12.0 + t2 / 720.0 : 1.0 / t2 - cos(0.5 * t) / (2.0 * t * sin(0.5 * t));
    R e[3] = {c == 0, c == 1, c == 2};
    R cr[3]; /* row c of [th]x */
    if (c == 0) { cr[0] = 0; cr[1] = -th[2]; cr[2] = th[1]; }
    else if (c == 1) { cr[0] = th[2]; cr[1] = 0; cr[2] = -th[0]; }
    else { cr[0] = -th[1]; cr[1] = th[0]; cr[2] = 0; }
    for (int x = 0; x < 3; ++x) row[x] = e[x] + 0.5 * cr[x] + k * (th[c] * th[x] - t2 * e[x]);
}

/* Joint limits (MJCF ranges, humanoid_phc.py:305-324) as unilateral rows on the exp-map joint
 * coordinates, speculative: a row is emitted within limit_margin + dt * (closing rate) of its bound.
 *  - component bounds inside (-pi, pi) (none in the SMPL MJCF, whose ranges are +-180 / +-720 deg):
 *    dof d of joint b with rate v = J_r^-1(q_b)_c . u_b, upper row -J_r^-1 row (gap upper - q_d),
 *    lower row +J_r^-1 row (gap q_d - lower);
 *  - the rotation angle |q_b| <= pi - LIMIT_PI_GUARD for every joint: a +-pi bound on an exp-map
 *    coordinate sits on the log map's branch cut (|q| = pi), where the coordinate wraps to -pi and
 *    the drive keeps spinning the joint (a +5 rad knee target). d|q|/dt = q^.u (q^ = q/|q| is a
 *    fixed vector of J_r^-1), so the row is -q^ over the joint's dofs, gap pi - guard - |q|.
 * Order: component rows in dof order (upper, then lower), then angle rows in joint order. */
#define LIMIT_PI_GUARD 0.02
/* Backstop when the limit rows lose (a limit against a deep self contact has no solution, and a
 * joint near 100 rad/s can cross the margin in one substep): the rotation angle never passes
 * pi - LIMIT_PI_GUARD / 2. nq = exp(q_old) (x) exp(dt u) before the log: its scalar part is
 * cos(angle / 2), negative when the rotation went past pi this substep (exp(q_old) has w >= 0 and
 * one substep turns by less than pi), in which case the log comes back on the far side with the
 * axis flipped -- that would reverse the joint's PD error and spin it. The angle is continued past
 * pi instead, then held at the cap on the joint's side with the outward rate q^ . u removed. */
static void limit_clamp(const R* nq, R* qv, R* u) {
    const R cap = M_PI - 0.5 * LIMIT_PI_GUARD;
    if (nq[3] >= cos(0.5 * cap)) return; /* inside the cap, not crossed: the common case */
    R t = sqrt(dot3(qv, qv));
    if (t < 1e-12) return;
    R dir[3] = {qv[0] / t, qv[1] / t, qv[2] / t};
    if (nq[3] < 0) {
        t = 2 * M_PI - t;
        for (int c = 0; c < 3; ++c) dir[c] = -dir[c];
    }
    if (t <= cap) return;
    for (int c = 0; c < 3; ++c) qv[c] = dir[c] * cap;
    R out = dot3(u, dir);
    if (out > 0)
        for (int c = 0; c < 3; ++c) u[c] -= out * dir[c];
}
/* the angle row of joint b: emitted (returns 1) within the margin of |q_b| = pi - guard */
static int angle_row(const he_sim_params* p, const env_state* s, int b, R* gap, R* dir) {
    const R* th = &s->q[3 * (b - 1)];
    const R* u = &s->u[3 * (b - 1)];
    R t = sqrt(dot3(th, th));
    if (t < 1e-6) return 0;
    for (int x = 0; x < 3; ++x) dir[x] = th[x] / t;
    *gap = M_PI - LIMIT_PI_GUARD - t;
    R closing = dot3(dir, u);
    return *gap < p->limit_margin + p->dt * (closing > 0 ? closing : 0);
}
static int gen_limits(const he_model* m, const he_sim_params* p, const env_state* s, contact* cs, int maxc, int* total) {
    int nc = 0;
    const R zero3[3] = {0, 0, 0}, up[3] = {0, 0, 1};
    const R cut = M_PI - LIMIT_PI_GUARD;
    for (int d = 0; d < ND; ++d) {
        int b = d / 3 + 1, c = d % 3;
        const R* th = &s->q[3 * (b - 1)];
        const R* u = &s->u[3 * (b - 1)];
        R row[3];
        jr_inv_row(th, c, row);
        R v = dot3(row, u);
        for (int side = 0; side < 2; ++side) {
            R bound = side == 0 ? m->dof_upper[d] : m->dof_lower[d];
            if (fabs(bound) >= cut) continue; /* held by the angle row */
            R gap = side == 0 ? bound - s->q[d] : s->q[d] - bound;
            R closing = side == 0 ? v : -v;
            if (gap < p->limit_margin + p->dt * (closing > 0 ? closing : 0)) {
                int slot = nc;
                nc = add_contact(cs, nc, maxc, total, b, -2, 1 + 2 * c + side, zero3, up, gap, 0.0);
                if (nc > slot)
                    for (int x = 0; x < 3; ++x) cs[slot].g[x] = side == 0 ? -row[x] : row[x];
            }
        }
    }
    for (int b = 1; b < NB; ++b) {
        R gap, dir[3];
        if (angle_row(p, s, b, &gap, dir)) {
            int slot = nc;
            nc = add_contact(cs, nc, maxc, total, b, -2, 7, zero3, up, gap, 0.0);
            if (nc > slot)
                for (int x = 0; x < 3; ++x) cs[slot].g[x] = -dir[x];
        }
    }
    return nc;
}

/* Solver rows of a slot set (limits 1; a body's terrain patch of k points k normal rows + 2
 * tangential + 1 torsional from k = 2; a self pair 3) */
/* diagnostic (tests/diag/anchor_study.py): PhysX-style two-anchor patch friction instead of the
 * centroid pair + torsional row. A terrain patch of >= 2 points gets 2 tangential rows at each of two
 * anchors -- its first point and the point farthest from it in the tangent plane -- each row bounded by
 * mu / 2 x the patch's normal impulses (the anchors share the patch's load); 1-point patches and self
 * pairs are unchanged. Off (0) in every test of the engine's physics. */
static int g_two_anchor = 0;
void ho_set_two_anchor(int on) { g_two_anchor = on; }
static int rows_of(const contact* cs, int nc) {
    int nr = 0, pos = 0; /* pos: the point's index in its body's terrain patch */
    for (int i = 0; i < nc; ++i) {
        if (cs[i].b1 != -1) { nr += cs[i].b1 == -2 ? 1 : 3; continue; }
        pos = (i > 0 && cs[i - 1].b1 == -1 && cs[i - 1].b0 == cs[i].b0) ? pos + 1 : 0;
        nr += pos == 0 ? 3 : (pos == 1 ? 2 + g_two_anchor : 1);
    }
    return nr;
}

/* Contact slots: joint limits, terrain (bodies in order, box corners deepest-first), self pairs.
 * All are generated (up to the oracle's own MAXC). When they exceed max_contacts slots or
 * HE_MAX_ROWS rows, the limits are kept and the contacts are taken deepest first (smallest gap,
 * ties in slot order), each one kept while its rows still fit (3 for a self pair or a body's first
 * terrain point, 2 for its second -- the normal and the patch's torsional row -- 1 after), and the
 * kept ones stay in slot order: the shallow speculative contacts go first, never a body's only
 * penetrating one. Returns the slots used; *total counts every contact generated. */
static int gen_all(const he_model* m, const he_sim_params* p, const kin* k, const env_state* s, int terrain_kind,
                   R mu, contact* cs, int* total, int* nlim_out);
/* diagnostic (tests/diag): the smallest gap among the dropped contacts of an env's last substep */
static __thread R g_drop_gap;
static float* g_drop_out;
void ho_set_drop_gap_out(float* out) { g_drop_out = out; }
/* diagnostic (tests): the friction bound weight of every solver row of the last substep, [N, HE_MAX_ROWS]
 * (mu for a tangential row, mu r_patch for a torsional one, 0 otherwise), in the cache's row order */
static float* g_roww_out;
void ho_set_row_weight_out(float* out) { g_roww_out = out; }
/* diagnostic (tests/diag): the gap of every solver row's contact of the last substep, [N, HE_MAX_ROWS] */
static float* g_rowgap_out;
void ho_set_row_gap_out(float* out) { g_rowgap_out = out; }
static int gen_contacts(const he_model* m, const he_sim_params* p, const kin* k, const env_state* s, int terrain_kind,
                        R mu, contact* cs, int* total) {
    int nlim = 0;
    g_drop_gap = INFINITY;
    int nc = gen_all(m, p, k, s, terrain_kind, mu, cs, total, &nlim);
    const int big = p->max_contacts > HE_MAX_CONTACTS; /* the oracle's own, larger capacity */
    const int maxc = p->max_contacts < MAXC ? p->max_contacts : MAXC;
    const int maxr = big ? MAXROW : HE_MAX_ROWS;
    if (nc <= maxc && rows_of(cs, nc) <= maxr) return nc;
    const int klim = nlim < maxc ? nlim : maxc; /* limits first, one row each */
    int order[MAXC], no = 0;
    for (int i = nlim; i < nc; ++i) {
        int j = no++; /* insertion by (gap, slot) */
        while (j > 0 && (cs[order[j - 1]].gap > cs[i].gap)) { order[j] = order[j - 1]; --j; }
        order[j] = i;
    }
    int kept[MAXC] = {0}, pc[NB] = {0};
    int rows = klim, slots = klim;
    for (int q = 0; q < no; ++q) {
        const int i = order[q];
        const int terr = cs[i].b1 == -1;
        const int cost = !terr ? 3 : (pc[cs[i].b0] == 0 ? 3 : (pc[cs[i].b0] == 1 ? 2 + g_two_anchor : 1));
        if (slots < maxc && rows + cost <= maxr) {
            kept[i] = 1;
            rows += cost;
            ++slots;
            if (terr) ++pc[cs[i].b0];
        }
    }
    int out = klim;
    for (int i = nlim; i < nc; ++i) {
        if (kept[i]) cs[out++] = cs[i];
        else if (cs[i].gap < g_drop_gap) g_drop_gap = cs[i].gap;
    }
    return out;
}

/* The solver rows of the kept slots (srow above), about the root origin o. */
static int build_rows(const contact* cs, int nc, const R* o, srow* rows) {
    int nr = 0;
    for (int i = 0; i < nc; ++i) {
        const contact* c = &cs[i];
        srow* r = &rows[nr];
        memset(r, 0, sizeof(*r));
        r->slot = i; r->kind = 0; r->n0 = nr; r->cnt = 1; r->b0 = c->b0; r->b1 = c->b1; r->key = c->key;
        if (c->b1 == -2) { ++nr; continue; } /* joint limit: its row is g over the joint's dofs */
        R xo[3] = {c->x[0] - o[0], c->x[1] - o[1], c->x[2] - o[2]};
        memcpy(r->dir, c->n, sizeof(r->dir));
        cross3(xo, c->n, r->rho);
        ++nr;
        const int terr = c->b1 == -1;
        if (terr && i + 1 < nc && cs[i + 1].b1 == -1 && cs[i + 1].b0 == c->b0) continue; /* not the patch's last point */
        int first = i;
        if (terr) while (first > 0 && cs[first - 1].b1 == -1 && cs[first - 1].b0 == c->b0) --first;
        const int cnt = i - first + 1;
        R np[3] = {0, 0, 0}, xp[3] = {0, 0, 0};
        for (int j = first; j <= i; ++j)
            for (int x = 0; x < 3; ++x) { np[x] += cs[j].n[x]; xp[x] += cs[j].x[x]; }
        const R nn = sqrt(dot3(np, np));
        for (int x = 0; x < 3; ++x) { np[x] /= nn; xp[x] /= cnt; }
        R t1[3], t2[3];
        friction_basis(np, t1, t2);
        R rp = 0;
        for (int j = first; j <= i; ++j) {
            R d[3] = {cs[j].x[0] - xp[0], cs[j].x[1] - xp[1], cs[j].x[2] - xp[2]};
            const R dn = dot3(d, np);
            R tg[3] = {d[0] - dn * np[0], d[1] - dn * np[1], d[2] - dn * np[2]};
            rp += sqrt(dot3(tg, tg));
        }
        rp /= cnt;
        R xpo[3] = {xp[0] - o[0], xp[1] - o[1], xp[2] - o[2]};
        if (g_two_anchor && terr && cnt >= 2) {
            int far = first;
            R best = -1;
            for (int j = first + 1; j <= i; ++j) {
                R d[3] = {cs[j].x[0] - cs[first].x[0], cs[j].x[1] - cs[first].x[1], cs[j].x[2] - cs[first].x[2]};
                const R dn = dot3(d, np);
                R tg[3] = {d[0] - dn * np[0], d[1] - dn * np[1], d[2] - dn * np[2]};
                const R dd = dot3(tg, tg);
                if (dd > best) { best = dd; far = j; }
            }
            const int anc[2] = {first, far};
            for (int a = 0; a < 2; ++a) {
                R xa[3] = {cs[anc[a]].x[0] - o[0], cs[anc[a]].x[1] - o[1], cs[anc[a]].x[2] - o[2]};
                for (int kd = 1; kd <= 2; ++kd) {
                    srow* f = &rows[nr++];
                    memset(f, 0, sizeof(*f));
                    f->slot = i; f->kind = kd; f->n0 = nr - 1 - (2 * a + kd - 1) - cnt;
                    f->cnt = cnt; f->b0 = c->b0; f->b1 = c->b1;
                    memcpy(f->dir, kd == 1 ? t1 : t2, sizeof(f->dir));
                    cross3(xa, f->dir, f->rho);
                    f->muw = 0.5 * c->mu;
                    f->key = (c->b0 | (1 << 5) | ((HE_KEY_PATCH - a) << 10)) | (kd << 14);
                }
            }
            continue;
        }
        const int nf = cnt >= 2 ? 3 : 2;
        for (int kd = 1; kd <= nf; ++kd) {
            srow* f = &rows[nr++];
            memset(f, 0, sizeof(*f));
            f->slot = i; f->kind = kd; f->n0 = nr - 1 - (kd - 1) - cnt; f->cnt = cnt; f->b0 = c->b0; f->b1 = c->b1;
            if (kd < 3) {
                memcpy(f->dir, kd == 1 ? t1 : t2, sizeof(f->dir));
                cross3(xpo, f->dir, f->rho);
                f->muw = c->mu;
            } else {
                memcpy(f->rho, np, sizeof(f->rho));
                f->muw = c->mu * rp;
            }
            f->key = (terr ? (c->b0 | (1 << 5) | (HE_KEY_PATCH << 10)) : c->key) | (kd << 14);
        }
    }
    return nr;
}
static int gen_all(const he_model* m, const he_sim_params* p, const kin* k, const env_state* s, int terrain_kind,
                   R mu, contact* cs, int* total, int* nlim_out) {
    int maxc = MAXC;
    *total = 0;
    int nc = p->joint_limits ? gen_limits(m, p, s, cs, maxc, total) : 0;
    *nlim_out = nc;
    R off = p->contact_offset;
    for (int b = 0; b < NB; ++b) {
        const float* g = m->geom_params[b];
        R n[3], x[3];
        if (m->geom_type[b] == HE_GEOM_SPHERE) {
            R l[3] = {g[0], g[1], g[2]}, c[3];
            body_point(k, b, l, c);
            R d = terrain_height(p, terrain_kind, c, n) - g[3];
            if (d < off) {
                for (int i = 0; i < 3; ++i) x[i] = c[i] - g[3] * n[i];
                nc = add_contact(cs, nc, maxc, total, b, -1, 0, x, n, d, mu);
            }
        } else if (m->geom_type[b] == HE_GEOM_CAPSULE) {
            for (int e = 0; e < 2; ++e) {
                R l[3] = {g[3 * e], g[3 * e + 1], g[3 * e + 2]}, c[3];
                body_point(k, b, l, c);
                R d = terrain_height(p, terrain_kind, c, n) - g[6];
                if (d < off) {
                    for (int i = 0; i < 3; ++i) x[i] = c[i] - g[6] * n[i];
                    nc = add_contact(cs, nc, maxc, total, b, -1, e, x, n, d, mu);
                }
            }
        } else {
            /* box corners, keep the 4 deepest (ties by corner index) */
            R bq[4] = {g[6], g[7], g[8], g[9]}, bm[3][3];
            qmat(bq, bm);
            R cx[8][3], cd[8], cn[8][3];
            int cand[8], ncand = 0;
            for (int ci = 0; ci < 8; ++ci) {
                R sgn[3] = {(ci & 1) ? 1.0 : -1.0, (ci & 2) ? 1.0 : -1.0, (ci & 4) ? 1.0 : -1.0};
                R lb[3] = {sgn[0] * g[3], sgn[1] * g[4], sgn[2] * g[5]}, lr[3];
                matvec(bm, lb, lr);
                R l[3] = {g[0] + lr[0], g[1] + lr[1], g[2] + lr[2]};
                body_point(k, b, l, cx[ci]);
                cd[ci] = terrain_height(p, terrain_kind, cx[ci], cn[ci]);
                if (cd[ci] < off) cand[ncand++] = ci;
            }
            /* the 4 deepest (ties by corner index), emitted in corner index order (resting
             * contacts keep their slots from one substep to the next) */
            int keep[8] = {0};
            for (int sel = 0; sel < 4 && ncand > 0; ++sel) {
                int best = 0;
                for (int j = 1; j < ncand; ++j)
                    if (cd[cand[j]] < cd[cand[best]]) best = j;
                keep[cand[best]] = 1;
                for (int j = best; j < ncand - 1; ++j) cand[j] = cand[j + 1];
                --ncand;
            }
            for (int ci = 0; ci < 8; ++ci)
                if (keep[ci]) nc = add_contact(cs, nc, maxc, total, b, -1, ci, cx[ci], cn[ci], cd[ci], mu);
        }
    }
    if (p->self_collision) {
        for (int pi = 0; pi < m->num_pairs; ++pi) {
            int i = m->pairs[pi][0], j = m->pairs[pi][1];
            R a0[3], a1[3], b0[3], b1[3], ri, rj, ci[3], cj[3];
            body_segment(m, k, i, a0, a1, &ri);
            body_segment(m, k, j, b0, b1, &rj);
            seg_seg(a0, a1, b0, b1, ci, cj);
            R d[3] = {ci[0] - cj[0], ci[1] - cj[1], ci[2] - cj[2]};
            R len = sqrt(dot3(d, d));
            R gap = len - ri - rj;
            if (gap < off) {
                R n[3];
                if (len > 1e-9) { n[0] = d[0] / len; n[1] = d[1] / len; n[2] = d[2] / len; }
                else { n[0] = 0; n[1] = 0; n[2] = 1; }
                R x[3];
                for (int c = 0; c < 3; ++c) x[c] = cj[c] + n[c] * (rj + 0.5 * gap);
                nc = add_contact(cs, nc, maxc, total, i, j, 0, x, n, gap, mu);
            }
        }
    }
    return nc;
}

/* ---------------------------------------------------------------- sparse LTDL (dense storage) */
static void ltdl_factor(R H[NG][NG], const int* lam) {
    for (int k = NG - 1; k >= 0; --k) {
        for (int i = lam[k]; i != -1; i = lam[i]) {
            R a = H[k][i] / H[k][k];
            for (int j = i; j != -1; j = lam[j]) H[i][j] -= a * H[k][j];
            H[k][i] = a;
        }
    }
}
static void ltdl_solve_LT(R H[NG][NG], const int* lam, R* y) { /* y <- L^-T y */
    for (int k = NG - 1; k >= 0; --k)
        for (int i = lam[k]; i != -1; i = lam[i]) y[i] -= H[k][i] * y[k];
}
static void ltdl_solve_L(R H[NG][NG], const int* lam, R* y) { /* y <- L^-1 y */
    for (int k = 0; k < NG; ++k)
        for (int i = lam[k]; i != -1; i = lam[i]) y[k] -= H[k][i] * y[i];
}

typedef struct step_out {
    R contact_force[NB][3];
    R dof_force[ND];
    int num_contacts;
    int dropped;          /* contacts generated past the capacity (last substep) */
    R residual;           /* max |complementarity residual| of the last substep's solve (m/s) */
    int sweeps;           /* Gauss-Seidel sweeps of the last substep's solve */
    int nr;               /* solver rows of the last substep */
    R muw[HE_MAX_ROWS];   /* their friction bound weights (0: a normal / limit row) */
    R gap[HE_MAX_ROWS];   /* their contact's gap (m; a limit row: its angle gap in rad) */
} step_out;

/* Warm-start cache: the previous solve's impulses by row key (PhysX warm-starts its solver from
 * the previous frame's impulses). A row whose key is found starts at the cached impulse instead
 * of 0. */
typedef struct warm_cache {
    int n;            /* rows */
    int key[MAXROW];  /* 16-bit row keys */
    R lam[MAXROW];
} warm_cache;

/* The contact row's velocity bias at separation `gap`: a speculative contact (gap >= 0) may close its gap
 * within the solve's step h, a penetrating one is pushed out at baumgarte * gap / dt, at most
 * max_depenetration_velocity (isaacgym_env.py:22), dt the physics step. TGS (solver_type 1) takes it
 * per position iteration (h = dt / iterations) from the separation its earlier iterations left; the
 * recovery rate of a penetration stays per physics step, whatever the iteration count (per iteration,
 * baumgarte * gap / h would push a 5 cm self-penetration out at 4x the PGS step's rate: under
 * saturated random actions that wedged limbs and launched 3 of 4096 standing bodies past 15 m/s,
 * tests/diag/tgs_study.py). */
static R contact_bias(const he_sim_params* p, R gap, R h, R dt) {
    return gap >= 0 ? gap / h : fmax(p->baumgarte * gap / dt, -p->max_depenetration_velocity);
}
/* diagnostic (tests/diag/tgs_study.py): TGS with the positions integrated once per position iteration
 * (h = dt / K, each with that iteration's velocity) instead of once with the iterations' mean velocity
 * (the engine's form). Off (0) in every test of the engine's physics. */
static int g_tgs_sequential = 0;
void ho_set_tgs_sequential(int on) { g_tgs_sequential = on; }
#define TGS_MAXIT 16

/* damping and the angular-velocity clamps of a generalized velocity (the body rotations of k) */
static void clamp_velocity(const he_model* m, const he_sim_params* p, const kin* k, R dt, R* unew) {
    /* angular damping and max angular velocity (asset options, humanoid_phc.py:212-213) */
    R damp = 1.0 / (1.0 + dt * p->angular_damping);
    for (int c = 0; c < 3; ++c) unew[c] *= damp;
    for (int d = 0; d < ND; ++d) unew[6 + d] *= damp;
    /* PhysX articulation joint maxJointVelocity (default 100 rad/s): each joint's relative rate */
    const R jmax = p->max_joint_velocity;
    for (int b = 1; b < NB; ++b) {
        R* w = &unew[6 + 3 * (b - 1)];
        R nrm = sqrt(dot3(w, w));
        if (nrm > jmax) { R sc = jmax / nrm; w[0] *= sc; w[1] *= sc; w[2] *= sc; }
    }
    /* max_angular_velocity (asset option, humanoid_phc.py:213; PxRigidBody maxAngularVelocity):
     * each link's WORLD angular velocity w_b = w_parent + R_b u_b, clamped link by link; the
     * joint rates are then re-derived from the clamped world rates, u_b = R_b^T (w'_b - w'_parent) */
    const R wmax = p->max_angular_velocity;
    R wo[NB][3], wc[NB][3];
    int any = 0;
    for (int c = 0; c < 3; ++c) wo[0][c] = unew[c];
    for (int b = 1; b < NB; ++b) {
        R r[3];
        matvec((R(*)[3])k->Rw[b], &unew[6 + 3 * (b - 1)], r);
        for (int c = 0; c < 3; ++c) wo[b][c] = wo[m->parents[b]][c] + r[c];
    }
    for (int b = 0; b < NB; ++b) {
        R nrm = sqrt(dot3(wo[b], wo[b])), sc = 1;
        if (nrm > wmax) { sc = wmax / nrm; any = 1; }
        for (int c = 0; c < 3; ++c) wc[b][c] = wo[b][c] * sc;
    }
    if (any) {
        for (int c = 0; c < 3; ++c) unew[c] = wc[0][c];
        for (int b = 1; b < NB; ++b) {
            const R* wp = wc[m->parents[b]];
            R rel[3] = {wc[b][0] - wp[0], wc[b][1] - wp[1], wc[b][2] - wp[2]};
            R* u = &unew[6 + 3 * (b - 1)];
            for (int c = 0; c < 3; ++c) u[c] = k->Rw[b][0][c] * rel[0] + k->Rw[b][1][c] * rel[1] + k->Rw[b][2][c] * rel[2];
        }
    }
}

/* semi-implicit position update over h with the velocity up (root: exp(h w) (x) q; ball joint:
 * log(exp(q) (x) exp(h u)) with the limit backstop, which also removes the outward rate from s->u) */
static void integrate_positions(const he_sim_params* p, env_state* s, const R* up, R h) {
    for (int c = 0; c < 3; ++c) s->root_pos[c] += h * up[3 + c];
    {
        R dw[3] = {h * up[0], h * up[1], h * up[2]}, dq[4], nq[4];
        qexp(dw, dq);
        qmul(dq, s->root_q, nq);
        qnormalize(nq);
        memcpy(s->root_q, nq, sizeof(nq));
    }
    for (int b = 1; b < NB; ++b) {
        R* qv = &s->q[3 * (b - 1)];
        const R* uj = &up[6 + 3 * (b - 1)];
        R ql[4], dq[4], nq[4], dw[3] = {h * uj[0], h * uj[1], h * uj[2]};
        qexp(qv, ql);
        qexp(dw, dq);
        qmul(ql, dq, nq);
        qnormalize(nq);
        qlog(nq, qv);
        if (p->joint_limits) limit_clamp(nq, qv, &s->u[3 * (b - 1)]);
    }
}

/* one substep; updates s in place */
/* Velocity-dependent + gravity bias at the velocities of state sv (the midpoint bias,
 * he_sim_params.bias_midpoint): the same RNEA as the substep's, with sv's body velocities. */
static void bias_at(const he_model* m, const topo* t, const he_sim_params* p, const env_state* sv, const kin* k,
                    const sinertia* I, R* bias) {
    static __thread kin kv;
    kinematics(m, t, sv, &kv);
    R Aacc[NB][6], F[NB][6];
    Aacc[0][0] = Aacc[0][1] = Aacc[0][2] = 0;
    {
        R vxw[3];
        cross3(sv->root_v, sv->root_w, vxw);
        for (int c = 0; c < 3; ++c) Aacc[0][3 + c] = vxw[c] - p->gravity[c];
    }
    for (int b = 1; b < NB; ++b) {
        int pb = m->parents[b];
        for (int i = 0; i < 6; ++i) Aacc[b][i] = Aacc[pb][i];
        for (int c = 0; c < 3; ++c) {
            R cr[6];
            crm(kv.V[b], k->S[t->body_dof0[b] + c], cr);
            R uu = sv->u[3 * (b - 1) + c];
            for (int i = 0; i < 6; ++i) Aacc[b][i] += cr[i] * uu;
        }
    }
    for (int b = 0; b < NB; ++b) {
        R IA[6], IV[6], x[6];
        si_apply(&I[b], Aacc[b], IA);
        si_apply(&I[b], kv.V[b], IV);
        crf(kv.V[b], IV, x);
        for (int i = 0; i < 6; ++i) F[b][i] = IA[i] + x[i];
    }
    for (int b = NB - 1; b > 0; --b) {
        int pb = m->parents[b];
        for (int i = 0; i < 6; ++i) F[pb][i] += F[b][i];
    }
    for (int i = 0; i < NG; ++i) {
        const R* S = k->S[i];
        const R* f = F[t->dof_body[i]];
        bias[i] = S[0] * f[0] + S[1] * f[1] + S[2] * f[2] + S[3] * f[3] + S[4] * f[4] + S[5] * f[5];
    }
}

/* J_r^T of solver row w (slot c) in generalized coordinates: a joint limit its row g over the joint's
 * dofs; a contact row S_i . (rho, dir) on the first body's chain, minus on the second's */
static void row_jacobian(const topo* t, const kin* k, const srow* w, const contact* c, R* z) {
    if (w->b1 == -2) { /* joint limit: the row over the joint's dofs */
        for (int i = 0; i < NG; ++i) z[i] = 0;
        for (int x = 0; x < 3; ++x) z[t->body_dof0[w->b0] + x] = c->g[x];
    } else {
        for (int i = 0; i < NG; ++i) {
            int bi = t->dof_body[i];
            R sgn = 0;
            if (t->is_anc[bi][w->b0]) sgn += 1;
            if (w->b1 >= 0 && t->is_anc[bi][w->b1]) sgn -= 1;
            const R* S = k->S[i];
            z[i] = sgn == 0 ? 0 : sgn * (S[0] * w->rho[0] + S[1] * w->rho[1] + S[2] * w->rho[2] + S[3] * w->dir[0] + S[4] * w->dir[1] + S[5] * w->dir[2]);
        }
    }
}

/* The step's dynamics at state s: kinematics k, the bodies' own spatial inertias I about o, the bias
 * forces (gravity + Coriolis / gyroscopic at s's velocities, RNEA with u_dot = 0) and the joint-space
 * inertia H (CRBA; no armature or drive terms). */
static void dynamics_terms(const he_model* m, const topo* t, const he_sim_params* p, const env_state* s,
                           const R* mass_scale, kin* k, sinertia* I, R* bias, R H[NG][NG]) {
    kinematics(m, t, s, k);
    sinertia Ic[NB];
    for (int b = 0; b < NB; ++b) body_inertia(m, k, b, mass_scale ? mass_scale[b] : 1.0, &I[b]);
    /* RNEA bias with u_dot = 0 and gravity (a_0 = -g) */
    R Aacc[NB][6], F[NB][6];
    Aacc[0][0] = Aacc[0][1] = Aacc[0][2] = 0;
    {
        R vxw[3];
        cross3(s->root_v, s->root_w, vxw);
        for (int c = 0; c < 3; ++c) Aacc[0][3 + c] = vxw[c] - p->gravity[c];
    }
    for (int b = 1; b < NB; ++b) {
        int pb = m->parents[b];
        for (int i = 0; i < 6; ++i) Aacc[b][i] = Aacc[pb][i];
        for (int c = 0; c < 3; ++c) {
            R cr[6];
            crm(k->V[b], k->S[t->body_dof0[b] + c], cr);
            R uu = s->u[3 * (b - 1) + c];
            for (int i = 0; i < 6; ++i) Aacc[b][i] += cr[i] * uu;
        }
    }
    for (int b = 0; b < NB; ++b) {
        R IA[6], IV[6], x[6];
        si_apply(&I[b], Aacc[b], IA);
        si_apply(&I[b], k->V[b], IV);
        crf(k->V[b], IV, x);
        for (int i = 0; i < 6; ++i) F[b][i] = IA[i] + x[i];
        Ic[b] = I[b];
    }
    for (int b = NB - 1; b > 0; --b) {
        int pb = m->parents[b];
        for (int i = 0; i < 6; ++i) F[pb][i] += F[b][i];
        si_add(&Ic[pb], &Ic[b]);
    }
    for (int i = 0; i < NG; ++i) {
        const R* S = k->S[i];
        const R* f = F[t->dof_body[i]];
        bias[i] = S[0] * f[0] + S[1] * f[1] + S[2] * f[2] + S[3] * f[3] + S[4] * f[4] + S[5] * f[5];
    }
    /* CRBA: H_ij = S_j . (Ic_{body(i)} S_i) for j ancestor-or-self of i */
    memset(H, 0, sizeof(R) * NG * NG);
    for (int i = 0; i < NG; ++i) {
        R IS[6];
        si_apply(&Ic[t->dof_body[i]], k->S[i], IS);
        for (int j = i; j != -1; j = t->dof_parent[j]) {
            const R* S = k->S[j];
            R v = S[0] * IS[0] + S[1] * IS[1] + S[2] * IS[2] + S[3] * IS[3] + S[4] * IS[4] + S[5] * IS[5];
            H[i][j] = v;
            H[j][i] = v;
        }
    }
}

static void substep(const he_model* m, const topo* t, const he_sim_params* p, env_state* s, const R* mass_scale,
                    R mu, int terrain_kind, step_out* out, warm_cache* ws) {
    static __thread kin k;
    static __thread R H[NG][NG];
    static __thread R Z[MAXROW][NG];
    static __thread R A[MAXROW][MAXROW];
    static __thread contact cs[MAXC];
    const R dt = p->dt;
    sinertia I[NB];
    R bias[NG];
    dynamics_terms(m, t, p, s, mass_scale, &k, I, bias, H);
    /* armature + implicit PD drives; a joint at its angle limit cannot give way to its drive, so
     * its effort check takes the drive torque at rest (no implicit relief) */
    R rhs[NG], coef[NG];
    int blocked[NB] = {0};
    if (p->joint_limits)
        for (int b = 1; b < NB; ++b) {
            R gap, dir[3];
            blocked[b] = angle_row(p, s, b, &gap, dir);
        }
    for (int i = 0; i < NG; ++i) { rhs[i] = -bias[i]; coef[i] = 0; }
    for (int d = 0; d < ND; ++d) {
        int g = 6 + d;
        H[g][g] += m->armature[d];
        R kp = m->stiffness[d] * p->kp_scale, kd = m->damping[d] * p->kd_scale;
        R err = s->target[d] - s->q[d];
        R u = s->u[d];
        R tau = kp * (err - dt * u) - kd * u;
        R lim = m->effort[d];
        /* Effort limit (dof_prop["effort"], humanoid_phc.py:324): PhysX solves the position drive
         * implicitly and clamps its impulse to maxForce dt. Restated per dof: the implicit step's
         * drive torque is estimated with the dof's own joint-space inertia h = H_gg (+ armature),
         * tau(u+) ~ tau - c dt (tau - bias) / (h + dt c) with c = dt kp + kd; when it exceeds the
         * limit, the whole drive (stiffness and damping) is scaled by lim / |tau(u+)|. The drive
         * stays an implicit spring-damper (unconditionally stable), only weaker; an explicit +-lim
         * torque without its damping drives light links into a bang-bang limit cycle. */
        R c = dt * kp + kd;
        R tau_i = blocked[d / 3 + 1] ? tau : tau - c * dt * (tau - bias[g]) / (H[g][g] + dt * c);
        if (fabs(tau_i) > lim) {
            R sc = lim / fabs(tau_i);
            kp *= sc;
            kd *= sc;
            tau *= sc;
        }
        H[g][g] += dt * (kd + dt * kp);
        out->dof_force[d] = tau; /* updated after the solve */
        rhs[g] += tau;
        coef[g] = dt * kp + kd; /* d tau / d u+ for the post-solve drive force */
    }
    ltdl_factor(H, t->dof_parent);
    R du[NG];
    for (int i = 0; i < NG; ++i) du[i] = dt * rhs[i];
    ltdl_solve_LT(H, t->dof_parent, du);
    for (int i = 0; i < NG; ++i) du[i] /= H[i][i];
    ltdl_solve_L(H, t->dof_parent, du);
    R u0[NG], uf[NG];
    for (int c = 0; c < 3; ++c) { u0[c] = s->root_w[c]; u0[3 + c] = s->root_v[c]; }
    for (int d = 0; d < ND; ++d) u0[6 + d] = s->u[d];
    for (int i = 0; i < NG; ++i) uf[i] = u0[i] + du[i];
    if (p->bias_midpoint) {
        /* The velocity-dependent bias (Coriolis, gyroscopic) taken at u0 alone is explicit: at
         * 1/120 s, stiff drives on light links under per-step random targets pump energy without
         * bound. It is taken again at the midpoint velocity um = (u0 + uf) / 2 of the
         * explicit step, and the free velocity corrected through the same factor:
         * uf += H^-1 dt (bias(u0) - bias(um)). One fixed-point pass of the implicit midpoint rule
         * (bias at (u0 + u+) / 2), which conserves the quadratic invariants of a free rigid body. */
        env_state sv = *s;
        R um[NG];
        for (int i = 0; i < NG; ++i) um[i] = 0.5 * (u0[i] + uf[i]);
        for (int c = 0; c < 3; ++c) { sv.root_w[c] = um[c]; sv.root_v[c] = um[3 + c]; }
        for (int d = 0; d < ND; ++d) sv.u[d] = um[6 + d];
        R b2[NG], dc[NG];
        bias_at(m, t, p, &sv, &k, I, b2);
        for (int i = 0; i < NG; ++i) dc[i] = dt * (bias[i] - b2[i]);
        ltdl_solve_LT(H, t->dof_parent, dc);
        for (int i = 0; i < NG; ++i) dc[i] /= H[i][i];
        ltdl_solve_L(H, t->dof_parent, dc);
        for (int i = 0; i < NG; ++i) uf[i] += dc[i];
    }
    /* contacts */
    int total = 0;
    int nc = gen_contacts(m, p, &k, s, terrain_kind, mu, cs, &total);
    out->num_contacts = nc;
    out->dropped = total - nc;
    out->residual = 0;
    out->nr = 0;
    memset(out->contact_force, 0, sizeof(out->contact_force));
    R unew[NG];
    memcpy(unew, uf, sizeof(unew));
    R upos[NG];          /* TGS: the velocity the positions advance by (the iterations' mean) */
    int have_upos = 0;
    static __thread R useq[TGS_MAXIT][NG]; /* TGS sequential diagnostic: each iteration's velocity */
    int nseq = 0;
    R lim_tau[ND];
    memset(lim_tau, 0, sizeof(lim_tau));
    if (nc > 0) {
        static __thread srow rows[MAXROW];
        const int nr = build_rows(cs, nc, k.o, rows);
        /* TGS (solver_type 1, isaacgym_env.py:16-18): K position iterations of h = dt / K, each one
         * sweep; a normal / limit row's separation advances by h J_r u_k after iteration k (the step's
         * rows, J linearised at its start) and its bias follows it. PGS: one step of dt. */
        const int tgs = p->solver_type == 2; /* the fixed-drive TGS form (study only) */
        const int K = tgs ? (p->solver_iterations > 0 ? (p->solver_iterations < TGS_MAXIT ? p->solver_iterations : TGS_MAXIT) : 1) : 1;
        const R h = tgs ? dt / K : dt;
        R brow[MAXROW], brow0[MAXROW], sep[MAXROW];
        for (int r = 0; r < nr; ++r) {
            const srow* w = &rows[r];
            const contact* c = &cs[w->slot];
            R* z = Z[r];
            row_jacobian(t, &k, w, c, z);
            R ju = 0;
            for (int i = 0; i < NG; ++i) ju += z[i] * uf[i];
            R bb = 0;
            if (w->kind == 0) bb = contact_bias(p, c->gap, h, dt);
            brow0[r] = ju;
            sep[r] = w->kind == 0 ? c->gap : 0;
            brow[r] = ju + bb;
            ltdl_solve_LT(H, t->dof_parent, z);
        }
        for (int r = 0; r < nr; ++r)
            for (int c2 = 0; c2 <= r; ++c2) {
                R acc = 0;
                for (int i = 0; i < NG; ++i) acc += Z[r][i] * Z[c2][i] / H[i][i];
                A[r][c2] = acc;
                A[c2][r] = acc;
            }
        if (g_probe_rel > 0) { /* sensitivity probe (above) */
            for (int r = 0; r < nr; ++r) {
                for (int c2 = 0; c2 <= r; ++c2) {
                    A[r][c2] *= 1.0 + g_probe_rel * probe_xi(r, c2);
                    A[c2][r] = A[r][c2];
                }
                const R f = 1.0 + g_probe_rel * probe_xi(r, MAXROW);
                brow[r] *= f;
                brow0[r] *= f;
            }
            ++g_probe_sub;
        }
        R lam[MAXROW];
        memset(lam, 0, sizeof(lam));
        if (ws && p->warm_start)
            for (int r = 0; r < nr; ++r)
                for (int j = 0; j < ws->n; ++j)
                    if (ws->key[j] == rows[r].key) {
                        lam[r] = ws->lam[j];
                        break;
                    }
        /* friction bound of row r from the current normal impulses of its patch */
#define PATCH_BOUND_OF(L_, r) ({ R b_ = 0; for (int k_ = 0; k_ < rows[r].cnt; ++k_) b_ += L_[rows[r].n0 + k_]; rows[r].muw * b_; })
#define PATCH_BOUND(r) PATCH_BOUND_OF(lam, r)
        int sweeps = 0;
        R lam_sum[MAXROW];
        static __thread R lamk[TGS_MAXIT][MAXROW]; /* each iteration's impulses (the sequential diagnostic) */
        memset(lam_sum, 0, sizeof(R) * nr);
        for (int it = 0; it < (tgs ? K : p->solver_iterations); ++it) {
            R lam_prev[MAXROW];
            memcpy(lam_prev, lam, sizeof(R) * nr);
            ++sweeps;
            for (int r = 0; r < nr; ++r) {
                R w = brow[r];
                for (int j = 0; j < nr; ++j) w += A[r][j] * lam[j];
                const R l = lam[r] - w / (A[r][r] + 1e-12);
                if (rows[r].kind == 0) {
                    lam[r] = l > 0 ? l : 0;
                } else {
                    const R bound = g_lagged_bounds ? PATCH_BOUND_OF(lam_prev, r) : PATCH_BOUND(r);
                    lam[r] = l > bound ? bound : (l < -bound ? -bound : l);
                }
            }
            if (tgs) { /* every iteration runs: they are sub-steps, not convergence sweeps */
                for (int r = 0; r < nr; ++r) { lam_sum[r] += lam[r]; lamk[it][r] = lam[r]; }
                if (it + 1 < K)
                    for (int r = 0; r < nr; ++r) {
                        if (rows[r].kind != 0) continue;
                        R v = brow0[r]; /* J_r u_k = J_r uf + (A lambda)_r */
                        for (int j = 0; j < nr; ++j) v += A[r][j] * lam[j];
                        sep[r] += h * v;
                        brow[r] = brow0[r] + contact_bias(p, sep[r], h, dt);
                    }
                continue;
            }
            /* converged: no row's velocity moved by more than solver_tolerance in this sweep
             * (|d lambda_r| A_rr); 0 runs every sweep */
            if (p->solver_tolerance > 0) {
                R mx = 0;
                for (int r = 0; r < nr; ++r) {
                    R dv = fabs(lam[r] - lam_prev[r]) * A[r][r];
                    if (dv > mx) mx = dv;
                }
                if (mx <= p->solver_tolerance) break;
            }
        }
        out->sweeps = sweeps;
        out->nr = nr < HE_MAX_ROWS ? nr : HE_MAX_ROWS;
        for (int r = 0; r < out->nr; ++r) {
            out->muw[r] = rows[r].kind == 0 ? 0 : rows[r].muw;
            out->gap[r] = cs[rows[r].slot].gap;
        }
        /* complementarity residual of the returned impulses: normal rows min(w, lambda) -> 0,
         * friction rows w = 0 inside the bound (or lambda on the bound) */
        for (int r = 0; r < nr; ++r) {
            R w = brow[r];
            for (int j = 0; j < nr; ++j) w += A[r][j] * lam[j];
            R res;
            if (rows[r].kind == 0) res = fmin(w, lam[r] * A[r][r]);
            else {
                const R bound = PATCH_BOUND(r);
                res = (lam[r] >= bound - 1e-12 && w < 0) || (lam[r] <= -bound + 1e-12 && w > 0) ? 0 : w;
            }
            if (fabs(res) > out->residual) out->residual = fabs(res);
        }
#undef PATCH_BOUND
        if (ws) {
            ws->n = nr;
            for (int r = 0; r < nr; ++r) {
                ws->key[r] = rows[r].key;
                ws->lam[r] = lam[r];
            }
        }
        R y[NG];
        memset(y, 0, sizeof(y));
        for (int r = 0; r < nr; ++r)
            if (lam[r] != 0) for (int i = 0; i < NG; ++i) y[i] += Z[r][i] * lam[r];
        for (int i = 0; i < NG; ++i) y[i] /= H[i][i];
        ltdl_solve_L(H, t->dof_parent, y);
        for (int i = 0; i < NG; ++i) unew[i] += y[i];
        if (tgs) { /* the positions' velocity: uf + M^-1 J^T (mean of the iterations' impulses) */
            memset(y, 0, sizeof(y));
            for (int r = 0; r < nr; ++r) {
                const R lb = lam_sum[r] / K;
                if (lb != 0) for (int i = 0; i < NG; ++i) y[i] += Z[r][i] * lb;
            }
            for (int i = 0; i < NG; ++i) y[i] /= H[i][i];
            ltdl_solve_L(H, t->dof_parent, y);
            for (int i = 0; i < NG; ++i) upos[i] = uf[i] + y[i];
            have_upos = 1;
            if (g_tgs_sequential) {
                nseq = K;
                for (int it = 0; it < K; ++it) {
                    memset(y, 0, sizeof(y));
                    for (int r = 0; r < nr; ++r)
                        if (lamk[it][r] != 0) for (int i = 0; i < NG; ++i) y[i] += Z[r][i] * lamk[it][r];
                    for (int i = 0; i < NG; ++i) y[i] /= H[i][i];
                    ltdl_solve_L(H, t->dof_parent, y);
                    for (int i = 0; i < NG; ++i) useq[it][i] = uf[i] + y[i];
                }
            }
        }
        for (int r = 0; r < nr; ++r) {
            const srow* w = &rows[r];
            if (w->b1 == -2) { /* a joint limit: a joint force (below), not a contact force */
                for (int x = 0; x < 3; ++x) lim_tau[3 * (w->b0 - 1) + x] += cs[w->slot].g[x] * lam[r] / dt;
                continue;
            }
            for (int x = 0; x < 3; ++x) { /* linear force of the row (a torsional row has none) */
                R f = lam[r] * w->dir[x] / dt;
                out->contact_force[w->b0][x] += f;
                if (w->b1 >= 0) out->contact_force[w->b1][x] -= f;
            }
        }
    } else if (ws) {
        ws->n = 0;
    }
    /* drive force actually applied: tau(u+) = tau_exp - (dt kp + kd)(u+ - u); then the joint-limit
     * force: dof_force is the joint's solver force, drive and limit constraints together (PhysX
     * articulations report the joint solver forces, PxArticulationCache::jointSolverForces; Isaac
     * Gym's dof-force sensor reads them -- unpinned here): the limit row g over the
     * joint's dofs with its impulse lambda adds g lambda / dt */
    for (int d = 0; d < ND; ++d) out->dof_force[d] -= coef[6 + d] * (unew[6 + d] - u0[6 + d]);
    for (int d = 0; d < ND; ++d) out->dof_force[d] += lim_tau[d];
    clamp_velocity(m, p, &k, dt, unew);
    /* write velocities + semi-implicit position update (TGS: by the iterations' mean velocity, or per
     * iteration in the sequential diagnostic) */
    for (int c = 0; c < 3; ++c) { s->root_w[c] = unew[c]; s->root_v[c] = unew[3 + c]; }
    for (int d = 0; d < ND; ++d) s->u[d] = unew[6 + d];
    if (nseq > 0) {
        for (int it = 0; it < nseq; ++it) {
            clamp_velocity(m, p, &k, dt, useq[it]);
            integrate_positions(p, s, useq[it], dt / nseq);
        }
    } else if (have_upos) {
        clamp_velocity(m, p, &k, dt, upos);
        integrate_positions(p, s, upos, dt);
    } else {
        integrate_positions(p, s, unew, dt);
    }
}

/* TGS (solver_type 1): sim_params.physx.solver_type = 1 with num_position_iterations = K and
 * num_velocity_iterations = 0 (isaacgym_env.py:16-18). One physics step of dt is K position iterations
 * of h = dt / K on the step's kinematics, factor and contact set (TGS keeps the step's contacts and
 * moves their separations; PhysX's TGS integrates the bodies once per position iteration):
 *   - the drives are implicit over one iteration (M~ = H + armature + h kd + h^2 kp, factored once),
 *     their error taken from the joint positions the earlier iterations reached;
 *   - iteration k: free velocity u + M~^-1 h (tau(q_k, u_k) - bias), one Gauss-Seidel sweep of the
 *     step's rows against it (bias from the row's separation, advanced by h J_r u_j of the earlier
 *     iterations), the impulse change applied, positions integrated by h with the damped and clamped
 *     velocity (the solver's velocity itself is not clamped; the last iteration's clamped one is the
 *     step's output);
 *   - the rows' impulses accumulate over the iterations (the step's total: the bounds and the reported
 *     forces, and the warm-start cache, as PGS's); each iteration's sweep starts from the accumulated
 *     impulses plus the previous iteration's change (the first: the previous step's total / K, its
 *     per-iteration share), as a small-step solver warm-starts each sub-step from the last; the drive
 *     force is the iterations' mean.
 * The velocity-dependent bias is taken at u0 for the whole step (bias_midpoint 0) or re-evaluated at
 * the start velocity of every second iteration with the step's kinematics (bias_midpoint 1,
 * g_bias_every above). */
/* TGS: the velocity-dependent bias is re-evaluated every g_bias_every-th position iteration (2: at
 * iterations 2, 4, ... with the step's start bias before): as stable under saturated random actions
 * as every iteration (airborne internal KE 759 against 768 J, the standing U(+-1) tail 7.9 m/s) and
 * with half the free-flight angular-momentum drift, at half the RNEA passes; every 4th (frozen over
 * the step) pumps energy (3.6 kJ). Study switch: ho_set_bias_every (tests/diag/tgs_study.py). */
static int g_bias_every = 2;
void ho_set_bias_every(int k) { g_bias_every = k < 1 ? 1 : k; }
static void substep_tgs(const he_model* m, const topo* t, const he_sim_params* p, env_state* s, const R* mass_scale,
                        R mu, int terrain_kind, step_out* out, warm_cache* ws) {
    static __thread kin k;
    static __thread R H[NG][NG];
    static __thread R Z[MAXROW][NG], J[MAXROW][NG];
    static __thread R A[MAXROW][MAXROW];
    static __thread contact cs[MAXC];
    static __thread srow rows[MAXROW];
    const R dt = p->dt;
    const int K = p->solver_iterations < 1 ? 1 : (p->solver_iterations > TGS_MAXIT ? TGS_MAXIT : p->solver_iterations);
    const R h = dt / K;
    sinertia I[NB];
    R bias[NG];
    dynamics_terms(m, t, p, s, mass_scale, &k, I, bias, H);
    /* drives implicit over one iteration; the effort limit as in substep() with the iteration's h
     * (PhysX clamps a drive's impulse per iteration to maxForce h) */
    int blocked[NB] = {0};
    if (p->joint_limits)
        for (int b = 1; b < NB; ++b) {
            R gap, dir[3];
            blocked[b] = angle_row(p, s, b, &gap, dir);
        }
    R kp[ND], kd[ND];
    for (int d = 0; d < ND; ++d) {
        const int g = 6 + d;
        H[g][g] += m->armature[d];
        R kpv = m->stiffness[d] * p->kp_scale, kdv = m->damping[d] * p->kd_scale;
        const R u = s->u[d];
        const R tau = kpv * ((s->target[d] - s->q[d]) - h * u) - kdv * u;
        const R c = h * kpv + kdv;
        const R tau_i = blocked[d / 3 + 1] ? tau : tau - c * h * (tau - bias[g]) / (H[g][g] + h * c);
        if (fabs(tau_i) > m->effort[d]) {
            const R sc = m->effort[d] / fabs(tau_i);
            kpv *= sc;
            kdv *= sc;
        }
        H[g][g] += h * (kdv + h * kpv);
        kp[d] = kpv;
        kd[d] = kdv;
    }
    ltdl_factor(H, t->dof_parent);
    /* the step's contact set and rows (at the step's start) */
    int total = 0;
    const int nc = gen_contacts(m, p, &k, s, terrain_kind, mu, cs, &total);
    out->num_contacts = nc;
    out->dropped = total - nc;
    out->residual = 0;
    out->nr = 0;
    memset(out->contact_force, 0, sizeof(out->contact_force));
    const int nr = nc > 0 ? build_rows(cs, nc, k.o, rows) : 0;
    R sep[MAXROW], lam[MAXROW], applied[MAXROW], guess[MAXROW], fprobe[MAXROW], wlast[MAXROW];
    for (int r = 0; r < nr; ++r) {
        row_jacobian(t, &k, &rows[r], &cs[rows[r].slot], J[r]);
        memcpy(Z[r], J[r], sizeof(R) * NG);
        ltdl_solve_LT(H, t->dof_parent, Z[r]);
        sep[r] = rows[r].kind == 0 ? cs[rows[r].slot].gap : 0;
        lam[r] = 0;
        applied[r] = 0;
        guess[r] = 0;
        fprobe[r] = 1;
    }
    for (int r = 0; r < nr; ++r)
        for (int c2 = 0; c2 <= r; ++c2) {
            R acc = 0;
            for (int i = 0; i < NG; ++i) acc += Z[r][i] * Z[c2][i] / H[i][i];
            A[r][c2] = acc;
            A[c2][r] = acc;
        }
    if (g_probe_rel > 0 && nr > 0) { /* sensitivity probe (see substep) */
        for (int r = 0; r < nr; ++r) {
            for (int c2 = 0; c2 <= r; ++c2) {
                A[r][c2] *= 1.0 + g_probe_rel * probe_xi(r, c2);
                A[c2][r] = A[r][c2];
            }
            fprobe[r] = 1.0 + g_probe_rel * probe_xi(r, MAXROW);
        }
        ++g_probe_sub;
    }
    /* warm start: each iteration's sweep starts from the accumulated impulses plus the previous
     * iteration's change (the first iteration: the previous step's last change, by row key) */
    if (ws && p->warm_start)
        for (int r = 0; r < nr; ++r)
            for (int j = 0; j < ws->n; ++j)
                if (ws->key[j] == rows[r].key) {
                    guess[r] = ws->lam[j] / K; /* the cache holds the previous step's total */
                    break;
                }
#define TGS_BOUND(r) ({ R b_ = 0; for (int k_ = 0; k_ < rows[r].cnt; ++k_) b_ += lam[rows[r].n0 + k_]; rows[r].muw * b_; })
    R u[NG];
    for (int c = 0; c < 3; ++c) { u[c] = s->root_w[c]; u[3 + c] = s->root_v[c]; }
    for (int d = 0; d < ND; ++d) u[6 + d] = s->u[d];
    env_state sw = *s; /* positions advance per iteration; s keeps the step's start */
    R dfor[ND];
    memset(dfor, 0, sizeof(dfor));
    R bias_it[NG];
    memcpy(bias_it, bias, sizeof(bias_it));
    for (int it = 0; it < K; ++it) {
        if (it > 0 && p->bias_midpoint && (it % g_bias_every) == 0) { /* the velocity-dependent bias at this iteration's velocity */
            env_state sv = *s;
            for (int c = 0; c < 3; ++c) { sv.root_w[c] = u[c]; sv.root_v[c] = u[3 + c]; }
            for (int d = 0; d < ND; ++d) sv.u[d] = u[6 + d];
            bias_at(m, t, p, &sv, &k, I, bias_it);
        }
        R y[NG];
        for (int i = 0; i < NG; ++i) y[i] = -h * bias_it[i];
        for (int d = 0; d < ND; ++d)
            y[6 + d] += h * (kp[d] * ((s->target[d] - sw.q[d]) - h * u[6 + d]) - kd[d] * u[6 + d]);
        ltdl_solve_LT(H, t->dof_parent, y);
        for (int i = 0; i < NG; ++i) y[i] /= H[i][i];
        ltdl_solve_L(H, t->dof_parent, y);
        R unew[NG];
        for (int i = 0; i < NG; ++i) unew[i] = u[i] + y[i]; /* the iteration's free velocity */
        if (nr > 0) {
            R brow[MAXROW];
            for (int r = 0; r < nr; ++r) {
                R ju = 0;
                for (int i = 0; i < NG; ++i) ju += J[r][i] * unew[i];
                brow[r] = ju * fprobe[r] + (rows[r].kind == 0 ? contact_bias(p, sep[r], h, dt) : 0);
            }
            for (int r = 0; r < nr; ++r) lam[r] = applied[r] + guess[r];
            for (int r = 0; r < nr; ++r) { /* one Gauss-Seidel sweep on the accumulated impulses */
                R w = brow[r];
                for (int j = 0; j < nr; ++j) w += A[r][j] * (lam[j] - applied[j]);
                const R l = lam[r] - w / (A[r][r] + 1e-12);
                if (rows[r].kind == 0) {
                    lam[r] = l > 0 ? l : 0;
                } else {
                    const R bound = TGS_BOUND(r);
                    lam[r] = l > bound ? bound : (l < -bound ? -bound : l);
                }
            }
            for (int r = 0; r < nr; ++r) { /* the rows' velocities after the sweep (the residual) */
                R w = brow[r];
                for (int j = 0; j < nr; ++j) w += A[r][j] * (lam[j] - applied[j]);
                wlast[r] = w;
            }
            memset(y, 0, sizeof(y));
            for (int r = 0; r < nr; ++r) {
                const R dl = lam[r] - applied[r];
                if (dl != 0) for (int i = 0; i < NG; ++i) y[i] += Z[r][i] * dl;
                applied[r] = lam[r];
                guess[r] = dl;
            }
            for (int i = 0; i < NG; ++i) y[i] /= H[i][i];
            ltdl_solve_L(H, t->dof_parent, y);
            for (int i = 0; i < NG; ++i) unew[i] += y[i];
            for (int r = 0; r < nr; ++r) /* separations after this iteration's motion */
                if (rows[r].kind == 0) {
                    R ju = 0;
                    for (int i = 0; i < NG; ++i) ju += J[r][i] * unew[i];
                    sep[r] += h * ju;
                }
        }
        /* the drive torque of the iteration, implicit at its end velocity */
        for (int d = 0; d < ND; ++d)
            dfor[d] += kp[d] * ((s->target[d] - sw.q[d]) - h * unew[6 + d]) - kd[d] * unew[6 + d];
        /* the positions advance by the damped, clamped velocity (damping over the step's dt; the
         * last iteration's is the step's output, with the limit backstop's outward rates removed);
         * the solver's own velocity stays as the sweeps left it (the rows' velocities J u are the
         * sweep's residuals, the kernel's delta form) */
        R ucl[NG];
        memcpy(ucl, unew, sizeof(ucl));
        clamp_velocity(m, p, &k, dt, ucl);
        for (int c = 0; c < 3; ++c) { sw.root_w[c] = ucl[c]; sw.root_v[c] = ucl[3 + c]; }
        for (int d = 0; d < ND; ++d) sw.u[d] = ucl[6 + d];
        integrate_positions(p, &sw, ucl, h); /* the limit backstop removes outward rates from sw.u */
        memcpy(u, unew, sizeof(u));
    }
    out->sweeps = K;
    out->nr = nr < HE_MAX_ROWS ? nr : HE_MAX_ROWS;
    R lim_tau[ND];
    memset(lim_tau, 0, sizeof(lim_tau));
    for (int r = 0; r < nr; ++r) {
        if (r < HE_MAX_ROWS) {
            out->muw[r] = rows[r].kind == 0 ? 0 : rows[r].muw;
            out->gap[r] = cs[rows[r].slot].gap;
        }
        R res; /* complementarity residual of the last iteration */
        if (rows[r].kind == 0) res = fmin(wlast[r], lam[r] * A[r][r]);
        else {
            const R bound = TGS_BOUND(r);
            res = (lam[r] >= bound - 1e-12 && wlast[r] < 0) || (lam[r] <= -bound + 1e-12 && wlast[r] > 0) ? 0 : wlast[r];
        }
        if (fabs(res) > out->residual) out->residual = fabs(res);
        const srow* w = &rows[r];
        if (w->b1 == -2) {
            for (int x = 0; x < 3; ++x) lim_tau[3 * (w->b0 - 1) + x] += cs[w->slot].g[x] * lam[r] / dt;
            continue;
        }
        for (int x = 0; x < 3; ++x) {
            const R f = lam[r] * w->dir[x] / dt;
            out->contact_force[w->b0][x] += f;
            if (w->b1 >= 0) out->contact_force[w->b1][x] -= f;
        }
    }
#undef TGS_BOUND
    if (ws) { /* the step's accumulated impulses: the next step's first guess is their per-iteration share */
        ws->n = nr;
        for (int r = 0; r < nr; ++r) {
            ws->key[r] = rows[r].key;
            ws->lam[r] = lam[r];
        }
    }
    for (int d = 0; d < ND; ++d) out->dof_force[d] = dfor[d] / K + lim_tau[d];
    *s = sw;
}

static void write_rb(const he_model* m, const topo* t, const env_state* s, float* rb) {
    kin k;
    kinematics(m, t, s, &k);
    for (int b = 0; b < NB; ++b) {
        R r[3] = {k.pw[b][0] - k.o[0], k.pw[b][1] - k.o[1], k.pw[b][2] - k.o[2]}, wxr[3];
        cross3(k.V[b], r, wxr);
        for (int c = 0; c < 3; ++c) {
            rb[b * 13 + c] = (float)k.pw[b][c];
            rb[b * 13 + 7 + c] = (float)(k.V[b][3 + c] + wxr[c]);
            rb[b * 13 + 10 + c] = (float)k.V[b][c];
        }
        for (int c = 0; c < 4; ++c) rb[b * 13 + 3 + c] = (float)k.qw[b][c];
    }
}

/* gym.simulate x num_simulate for n envs: num_simulate x p->substeps physics steps of
 * p->dt / p->substeps (gymapi.SimParams.substeps, Isaac Gym default 2). root_states [N,13], dof_state [N,69,2] (in/out),
 * targets [N,69]; outputs rb_state [N,24,13], contact_forces [N,24,3], dof_force [N,69],
 * num_contacts [N] (nullable). mass_scale [N,24], friction [N], terrain_kind [N] nullable.
 * cache [N,HE_CACHE_WORDS] (in/out, nullable: cold solves), dropped [N], residual [N] and
 * sweeps [N] (out, nullable): contacts past the capacity, the solve's residual and its sweep count,
 * all of the last substep. */
void ho_physics_step(const he_model* m, const he_sim_params* p, int n, float* root_states, float* dof_state,
                     const float* targets, int num_simulate, float* rb_state, float* contact_forces, float* dof_force,
                     int32_t* num_contacts, const float* mass_scale, const float* friction, const int32_t* terrain_kind,
                     float* cache, int32_t* dropped, float* residual, int32_t* sweeps) {
    topo t;
    build_topo(m, &t);
    he_sim_params ps = *p; /* the physics step's parameters: dt / substeps */
    const int nsub = p->substeps > 0 ? p->substeps : 1;
    ps.dt = p->dt / nsub;
    const int substeps = num_simulate * nsub;
    p = &ps;
#pragma omp parallel for schedule(dynamic, 4)
    for (int e = 0; e < n; ++e) {
        env_state s;
        float* rs = root_states + (size_t)e * 13;
        for (int c = 0; c < 3; ++c) { s.root_pos[c] = rs[c]; s.root_v[c] = rs[7 + c]; s.root_w[c] = rs[10 + c]; }
        for (int c = 0; c < 4; ++c) s.root_q[c] = rs[3 + c];
        for (int d = 0; d < ND; ++d) {
            s.q[d] = dof_state[((size_t)e * ND + d) * 2];
            s.u[d] = dof_state[((size_t)e * ND + d) * 2 + 1];
            s.target[d] = targets[(size_t)e * ND + d];
        }
        R ms[NB];
        if (mass_scale) for (int b = 0; b < NB; ++b) ms[b] = mass_scale[(size_t)e * NB + b];
        R mu = friction ? friction[e] : p->friction;
        int tk = (p->terrain && terrain_kind) ? terrain_kind[e] : 0;
        warm_cache ws;
        ws.n = 0;
        float* cw = cache ? cache + (size_t)e * HE_CACHE_WORDS : NULL;
        if (cw && p->warm_start && memcmp(cw, rs, 7 * sizeof(float)) == 0) {
            int32_t nn;
            memcpy(&nn, cw + 7, 4);
            ws.n = nn < 0 ? 0 : (nn > HE_MAX_ROWS ? HE_MAX_ROWS : nn);
            for (int j = 0; j < ws.n; ++j) {
                uint32_t kw;
                memcpy(&kw, cw + HE_CACHE_KEYS + j / 2, 4);
                ws.key[j] = (int)((kw >> (16 * (j & 1))) & 0xFFFFu);
                ws.lam[j] = cw[HE_CACHE_LAMBDA + j];
            }
        }
        step_out out;
        memset(&out, 0, sizeof(out));
        g_probe_env = e;
        g_probe_sub = 0;
        for (int it = 0; it < substeps; ++it)
            (p->solver_type == 1 ? substep_tgs : substep)(m, &t, p, &s, mass_scale ? ms : NULL, mu, tk, &out, &ws);
        for (int c = 0; c < 3; ++c) { rs[c] = (float)s.root_pos[c]; rs[7 + c] = (float)s.root_v[c]; rs[10 + c] = (float)s.root_w[c]; }
        for (int c = 0; c < 4; ++c) rs[3 + c] = (float)s.root_q[c];
        for (int d = 0; d < ND; ++d) {
            dof_state[((size_t)e * ND + d) * 2] = (float)s.q[d];
            dof_state[((size_t)e * ND + d) * 2 + 1] = (float)s.u[d];
            dof_force[(size_t)e * ND + d] = (float)out.dof_force[d];
        }
        write_rb(m, &t, &s, rb_state + (size_t)e * NB * 13);
        for (int b = 0; b < NB; ++b)
            for (int c = 0; c < 3; ++c) contact_forces[((size_t)e * NB + b) * 3 + c] = (float)out.contact_force[b][c];
        if (num_contacts) num_contacts[e] = out.num_contacts;
        if (dropped) dropped[e] = out.dropped;
        if (residual) residual[e] = (float)out.residual;
        if (sweeps) sweeps[e] = out.sweeps;
        if (g_drop_out) g_drop_out[e] = (float)g_drop_gap;
        if (g_roww_out)
            for (int r = 0; r < HE_MAX_ROWS; ++r) g_roww_out[(size_t)e * HE_MAX_ROWS + r] = r < out.nr ? (float)out.muw[r] : 0.f;
        if (g_rowgap_out)
            for (int r = 0; r < HE_MAX_ROWS; ++r) g_rowgap_out[(size_t)e * HE_MAX_ROWS + r] = r < out.nr ? (float)out.gap[r] : 0.f;
        if (cw) {
            memset(cw, 0, HE_CACHE_WORDS * sizeof(float));
            if (p->warm_start) {
                memcpy(cw, rs, 7 * sizeof(float));
                int32_t nn = ws.n > HE_MAX_ROWS ? HE_MAX_ROWS : ws.n; /* the oracle's larger capacity: truncated */
                memcpy(cw + 7, &nn, 4);
                for (int j = 0; j < nn; ++j) {
                    uint32_t kw;
                    memcpy(&kw, cw + HE_CACHE_KEYS + j / 2, 4);
                    kw |= ((uint32_t)ws.key[j] & 0xFFFFu) << (16 * (j & 1));
                    memcpy(cw + HE_CACHE_KEYS + j / 2, &kw, 4);
                    cw[HE_CACHE_LAMBDA + j] = (float)ws.lam[j];
                }
            }
        }
    }
}

/* kinematics only: rigid-body state of given generalized states (used by tests) */
void ho_forward_kinematics(const he_model* m, int n, const float* root_states, const float* dof_state, float* rb_state) {
    topo t;
    build_topo(m, &t);
    for (int e = 0; e < n; ++e) {
        env_state s;
        const float* rs = root_states + (size_t)e * 13;
        for (int c = 0; c < 3; ++c) { s.root_pos[c] = rs[c]; s.root_v[c] = rs[7 + c]; s.root_w[c] = rs[10 + c]; }
        for (int c = 0; c < 4; ++c) s.root_q[c] = rs[3 + c];
        for (int d = 0; d < ND; ++d) { s.q[d] = dof_state[((size_t)e * ND + d) * 2]; s.u[d] = dof_state[((size_t)e * ND + d) * 2 + 1]; }
        write_rb(m, &t, &s, rb_state + (size_t)e * NB * 13);
    }
}

/* total mechanical quantities for invariant tests: linear momentum [3], angular momentum about
 * the world origin [3], kinetic energy, potential energy (gravity). */
void ho_momentum_energy(const he_model* m, const he_sim_params* p, int n, const float* root_states,
                        const float* dof_state, double* out /* [N,8] */) {
    topo t;
    build_topo(m, &t);
    for (int e = 0; e < n; ++e) {
        env_state s;
        const float* rs = root_states + (size_t)e * 13;
        for (int c = 0; c < 3; ++c) { s.root_pos[c] = rs[c]; s.root_v[c] = rs[7 + c]; s.root_w[c] = rs[10 + c]; }
        for (int c = 0; c < 4; ++c) s.root_q[c] = rs[3 + c];
        for (int d = 0; d < ND; ++d) { s.q[d] = dof_state[((size_t)e * ND + d) * 2]; s.u[d] = dof_state[((size_t)e * ND + d) * 2 + 1]; }
        kin k;
        kinematics(m, &t, &s, &k);
        R P[6] = {0}, ke = 0, pe = 0;
        for (int b = 0; b < NB; ++b) {
            sinertia I;
            body_inertia(m, &k, b, 1.0, &I);
            R h[6];
            si_apply(&I, k.V[b], h); /* momentum about o: (L_o, p) */
            for (int i = 0; i < 6; ++i) P[i] += h[i];
            ke += 0.5 * (h[0] * k.V[b][0] + h[1] * k.V[b][1] + h[2] * k.V[b][2] + h[3] * k.V[b][3] + h[4] * k.V[b][4] + h[5] * k.V[b][5]);
            R com_z = k.o[2] + I.h[2] / I.m;
            pe += -I.m * p->gravity[2] * com_z;
        }
        /* angular momentum about world origin: L_0 = L_o + o x p */
        R oxp[3];
        cross3(k.o, P + 3, oxp);
        double* o = out + (size_t)e * 8;
        o[0] = P[3]; o[1] = P[4]; o[2] = P[5];
        o[3] = P[0] + oxp[0]; o[4] = P[1] + oxp[1]; o[5] = P[2] + oxp[2];
        o[6] = ke; o[7] = pe;
    }
}

/* The step's dynamics terms for the independent pins (tests/test_independent_dynamics.py): the CRBA
 * joint-space inertia H [N,75,75] (no armature) and the RNEA bias [N,75] (gravity + Coriolis /
 * gyroscopic at the state's velocities), as dynamics_terms computes them for substep. */
void ho_dynamics_terms(const he_model* m, const he_sim_params* p, int n, const float* root_states,
                       const float* dof_state, double* H_out, double* bias_out) {
    topo t;
    build_topo(m, &t);
    for (int e = 0; e < n; ++e) {
        env_state s;
        const float* rs = root_states + (size_t)e * 13;
        for (int c = 0; c < 3; ++c) { s.root_pos[c] = rs[c]; s.root_v[c] = rs[7 + c]; s.root_w[c] = rs[10 + c]; }
        for (int c = 0; c < 4; ++c) s.root_q[c] = rs[3 + c];
        for (int d = 0; d < ND; ++d) { s.q[d] = dof_state[((size_t)e * ND + d) * 2]; s.u[d] = dof_state[((size_t)e * ND + d) * 2 + 1]; }
        static __thread kin k;
        static __thread R H[NG][NG];
        sinertia I[NB];
        R bias[NG];
        dynamics_terms(m, &t, p, &s, NULL, &k, I, bias, H);
        memcpy(H_out + (size_t)e * NG * NG, H, sizeof(R) * NG * NG);
        memcpy(bias_out + (size_t)e * NG, bias, sizeof(R) * NG);
    }
}

/* J^T of a contact row on body b at world point x along direction d (the terrain case of
 * row_jacobian: rho = (x - o) x d over b's chain), per env: z [N,75] */
void ho_point_jacobian(const he_model* m, int n, const float* root_states, const float* dof_state, const int* body,
                       const double* x, const double* d, double* z_out) {
    topo t;
    build_topo(m, &t);
    for (int e = 0; e < n; ++e) {
        env_state s;
        const float* rs = root_states + (size_t)e * 13;
        for (int c = 0; c < 3; ++c) { s.root_pos[c] = rs[c]; s.root_v[c] = rs[7 + c]; s.root_w[c] = rs[10 + c]; }
        for (int c = 0; c < 4; ++c) s.root_q[c] = rs[3 + c];
        for (int q = 0; q < ND; ++q) { s.q[q] = dof_state[((size_t)e * ND + q) * 2]; s.u[q] = dof_state[((size_t)e * ND + q) * 2 + 1]; }
        kin k;
        kinematics(m, &t, &s, &k);
        srow w;
        memset(&w, 0, sizeof(w));
        w.b0 = body[e];
        w.b1 = -1;
        const R r[3] = {x[3 * e] - k.o[0], x[3 * e + 1] - k.o[1], x[3 * e + 2] - k.o[2]};
        for (int c = 0; c < 3; ++c) w.dir[c] = d[3 * e + c];
        cross3(r, w.dir, w.rho);
        contact cdummy;
        memset(&cdummy, 0, sizeof(cdummy));
        row_jacobian(&t, &k, &w, &cdummy, z_out + (size_t)e * NG);
    }
}

/* J_r^-1(th) [3x3] row by row as the limit rows use it (jr_inv_row), for the independent pin */
void ho_jr_inv(const double* th, double* out) {
    for (int c = 0; c < 3; ++c) jr_inv_row(th, c, out + 3 * c);
}
