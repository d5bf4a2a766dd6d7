/*
 * he_oracle.c -- TEST INFRASTRUCTURE ONLY. CPU restatement used as the parity checker for
 * libhumanoid_engine.so; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load it. It is never on the product path.
 *
 * Part 1 (imitation): restates the reference's pure-torch code
 *   motion_lib.py:549-673 (get_motion_state, _calc_frame_blend, _local_rotation_to_dof_smpl),
 *   motion_lib.py:526-535 (sample_time_interval), torch_utils.py:54-408 (quaternion library),
 *   envs/common.py:22-176 (self/task observations), :270-364 (reward, reset),
 *   envs/humanoid_phc.py:1230-1335 (reward/reset glue, power reward), :937-1123 (obs glue),
 *   :694-780, 901-931 (reset-to-reference-state).
 *   Pinned by the tests/golden fixtures produced by running the reference itself (tools/gen_golden.py).
 *   Math is double precision; the frame-index arithmetic follows the reference's float32 ops
 *   exactly (the oracle is compiled with -ffp-contract=off).
 *
 * Part 2 (physics, A1-A4, he_oracle_physics.c): the engine's own articulated-body specification
 *   (DESIGN.md §5). Isaac Gym/PhysX is closed and absent: PHYSICS PARITY VS PHYSX IS
 *   UNPINNED. This fp64 scalar implementation is the reference the HIP kernel is checked against,
 *   and is itself pinned by the invariant tests of tests/test_physics_invariants.py (free fall,
 *   momentum / angular momentum / energy drift, ballistic CoM, dt refinement, PD stand-still,
 *   penetration) and tests/test_limits_contacts.py (joint limits, overflow reduction, warm start).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/humanoid_engine.h"

typedef double R;
#define NB HE_NUM_BODIES
#define ND HE_NUM_DOF
#define NG HE_NUM_GEN

/* ------------------------------------------------------------------------------------- */
/* small vector / quaternion helpers (xyzw)                                                */
/* ------------------------------------------------------------------------------------- */
static inline void v3_sub(const R* a, const R* b, R* o) { o[0] = a[0] - b[0]; o[1] = a[1] - b[1]; o[2] = a[2] - b[2]; }
static inline void v3_add(const R* a, const R* b, R* o) { o[0] = a[0] + b[0]; o[1] = a[1] + b[1]; o[2] = a[2] + b[2]; }
static inline R v3_dot(const R* a, const R* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void v3_cross(const R* a, const R* b, R* o) {
    R x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}
static inline R v3_norm(const R* a) { return sqrt(v3_dot(a, a)); }

/* torch_utils.py:54-75 (8-multiplication form) */
static void q_mul(const R* a, const R* b, R* o) {
    R x1 = a[0], y1 = a[1], z1 = a[2], w1 = a[3], x2 = b[0], y2 = b[1], z2 = b[2], w2 = b[3];
    R ww = (z1 + x1) * (x2 + y2), yy = (w1 - y1) * (w2 + z2), zz = (w1 + y1) * (w2 - z2);
    R xx = ww + yy + zz, qq = 0.5 * (xx + (z1 - x1) * (x2 - y2));
    R w = qq - ww + (z1 - y1) * (y2 - z2);
    R x = qq - xx + (x1 + w1) * (x2 + w2);
    R y = qq - yy + (w1 - x1) * (y2 + z2);
    R z = qq - zz + (z1 + y1) * (w2 - x2);
    o[0] = x; o[1] = y; o[2] = z; o[3] = w;
}
static inline void q_conj(const R* a, R* o) { o[0] = -a[0]; o[1] = -a[1]; o[2] = -a[2]; o[3] = a[3]; }
/* torch_utils.py:273-281 my_quat_rotate */
static void q_rot(const R* q, const R* v, R* o) {
    R w = q[3];
    R s = 2.0 * w * w - 1.0;
    R c[3];
    v3_cross(q, v, c);
    R d = v3_dot(q, v);
    for (int i = 0; i < 3; ++i) o[i] = v[i] * s + c[i] * w * 2.0 + q[i] * d * 2.0;
}
/* torch_utils.py:284-297 */
static void q_tan_norm(const R* q, R* o) {
    static const R ex[3] = {1, 0, 0}, ez[3] = {0, 0, 1};
    q_rot(q, ex, o);
    q_rot(q, ez, o + 3);
}
/* torch_utils.py:49-51 */
static inline R normalize_angle(R x) { return atan2(sin(x), cos(x)); }
/* torch_utils.py:85-106: returns angle; axis optional */
static R q_angle_axis(const R* q, R* axis) {
    R w = q[3];
    R s = sqrt(1 - w * w);
    R angle = normalize_angle(2 * acos(w));
    int mask = fabs(s) > 1e-5; /* NaN -> false */
    if (axis) {
        if (mask) { axis[0] = q[0] / s; axis[1] = q[1] / s; axis[2] = q[2] / s; }
        else { axis[0] = 0; axis[1] = 0; axis[2] = 1; }
    }
    return mask ? angle : 0.0;
}
/* torch_utils.py:143-150 */
static void q_to_exp_map(const R* q, R* o) {
    R ax[3];
    R a = q_angle_axis(q, ax);
    o[0] = a * ax[0]; o[1] = a * ax[1]; o[2] = a * ax[2];
}
/* torch_utils.py:353-365 exp_map_to_quat */
static void exp_map_to_q(const R* e, R* o) {
    R angle = v3_norm(e);
    R axis[3] = {e[0] / angle, e[1] / angle, e[2] / angle};
    R an = normalize_angle(angle);
    if (!(fabs(an) > 1e-5)) { an = 0; axis[0] = 0; axis[1] = 0; axis[2] = 1; }
    R n = v3_norm(axis);
    if (n < 1e-9) n = 1e-9;
    R s = sin(an / 2), c = cos(an / 2);
    R q[4] = {axis[0] / n * s, axis[1] / n * s, axis[2] / n * s, c};
    R qn = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    if (qn < 1e-9) qn = 1e-9;
    for (int i = 0; i < 4; ++i) o[i] = q[i] / qn;
}
/* torch_utils.py:109-131, evaluated in float32 with torch's operation order: the reference's
 * slerp is ill-conditioned at small angles (float32 acos(c) near 1 against sqrt(1-c*c)), so
 * double evaluation would differ from it by up to ~1e-4; the branch tests are discontinuous. */
static void q_slerp_f(const float* q0f, const float* q1f, R t, R* o) {
    float cf = q0f[0] * q1f[0];
    cf = cf + q0f[1] * q1f[1];
    cf = cf + q0f[2] * q1f[2];
    cf = cf + q0f[3] * q1f[3];
    float q1[4];
    for (int i = 0; i < 4; ++i) q1[i] = cf < 0.0f ? -q1f[i] : q1f[i];
    cf = fabsf(cf);
    float half = acosf(cf);
    float sf = sqrtf(1.0f - cf * cf);
    float tf = (float)t;
    float ra = sinf((1.0f - tf) * half) / sf, rb = sinf(tf * half) / sf;
    for (int i = 0; i < 4; ++i) {
        float a = ra * q0f[i], b = rb * q1[i];
        o[i] = a + b;
    }
    if (fabsf(sf) < 0.001f) for (int i = 0; i < 4; ++i) { float a = 0.5f * q0f[i], b = 0.5f * q1[i]; o[i] = a + b; }
    if (cf >= 1.0f) for (int i = 0; i < 4; ++i) o[i] = q0f[i];
}
static void q_slerp(const R* q0, const R* q1, R t, R* o) {
    float a[4], b[4];
    for (int i = 0; i < 4; ++i) { a[i] = (float)q0[i]; b[i] = (float)q1[i]; }
    q_slerp_f(a, b, t, o);
}
/* torch_utils.py:368-408 */
static R calc_heading(const R* q) {
    static const R ex[3] = {1, 0, 0};
    R d[3];
    q_rot(q, ex, d);
    return atan2(d[1], d[0]);
}
static void heading_quat(R heading, R* o) { /* quat_from_angle_axis(heading, z) */
    R s = sin(heading / 2), c = cos(heading / 2);
    R n = sqrt(s * s + c * c);
    if (n < 1e-9) n = 1e-9;
    o[0] = 0; o[1] = 0; o[2] = s / n; o[3] = c / n;
}

/* exported primitives for the golden tests (float in / float out, n items) */
void ho_quat_prims(int n, const float* q, const float* r, const float* v, const float* e, const float* t,
                   float* mul, float* rot, float* tan_norm, float* angle, float* axis, float* expmap,
                   float* exp2q, float* slerp, float* heading, float* hq, float* hqi) {
    for (int i = 0; i < n; ++i) {
        R a[4], b[4], vv[3], ee[3], o[6];
        for (int k = 0; k < 4; ++k) { a[k] = q[4 * i + k]; b[k] = r[4 * i + k]; }
        for (int k = 0; k < 3; ++k) { vv[k] = v[3 * i + k]; ee[k] = e[3 * i + k]; }
        q_mul(a, b, o); for (int k = 0; k < 4; ++k) mul[4 * i + k] = (float)o[k];
        q_rot(a, vv, o); for (int k = 0; k < 3; ++k) rot[3 * i + k] = (float)o[k];
        q_tan_norm(a, o); for (int k = 0; k < 6; ++k) tan_norm[6 * i + k] = (float)o[k];
        R ax[3];
        angle[i] = (float)q_angle_axis(a, ax);
        for (int k = 0; k < 3; ++k) axis[3 * i + k] = (float)ax[k];
        q_to_exp_map(a, o); for (int k = 0; k < 3; ++k) expmap[3 * i + k] = (float)o[k];
        exp_map_to_q(ee, o); for (int k = 0; k < 4; ++k) exp2q[4 * i + k] = (float)o[k];
        q_slerp(a, b, t[i], o); for (int k = 0; k < 4; ++k) slerp[4 * i + k] = (float)o[k];
        R h = calc_heading(a);
        heading[i] = (float)h;
        heading_quat(h, o); for (int k = 0; k < 4; ++k) hq[4 * i + k] = (float)o[k];
        heading_quat(-h, o); for (int k = 0; k < 4; ++k) hqi[4 * i + k] = (float)o[k];
    }
}

/* ------------------------------------------------------------------------------------- */
/* Part 1: motion library sampling + imitation reward / reset / observations               */
/* ------------------------------------------------------------------------------------- */
typedef struct ho_motion {
    const float *gts, *grs, *lrs, *gvs, *gavs, *dvs;
    const int64_t *length_starts, *num_frames;
    const float *lengths, *dt;
} ho_motion;

typedef struct mstate {
    R pos[NB][3], rot[NB][4], vel[NB][3], ang[NB][3];
    R dof_pos[ND], dof_vel[ND];
} mstate;

/* motion_lib.py:655-665, float32 exactly as torch computes it */
static void frame_blend(float time, float len, int64_t nf, float dt, int64_t* f0, int64_t* f1, float* blend) {
    float phase = time / len;
    phase = phase < 0.0f ? 0.0f : (phase > 1.0f ? 1.0f : phase);
    if (time < 0) time = 0;
    int64_t i0 = (int64_t)(phase * (float)(nf - 1));
    int64_t i1 = i0 + 1 < nf - 1 ? i0 + 1 : nf - 1;
    float b = (time - (float)i0 * dt) / dt;
    b = b < 0.0f ? 0.0f : (b > 1.0f ? 1.0f : b);
    *f0 = i0; *f1 = i1; *blend = b;
}

/* motion_lib.py:549-626 */
static void motion_eval(const ho_motion* M, int64_t id, float time, const float* offset, int want_dof, mstate* s) {
    int64_t f0, f1;
    float bl;
    frame_blend(time, M->lengths[id], M->num_frames[id], M->dt[id], &f0, &f1, &bl);
    int64_t g0 = f0 + M->length_starts[id], g1 = f1 + M->length_starts[id];
    R b = bl, a = 1.0 - b;
    for (int j = 0; j < NB; ++j) {
        for (int k = 0; k < 3; ++k) {
            s->pos[j][k] = a * M->gts[(g0 * NB + j) * 3 + k] + b * M->gts[(g1 * NB + j) * 3 + k] + (offset ? offset[k] : 0.0);
            s->vel[j][k] = a * M->gvs[(g0 * NB + j) * 3 + k] + b * M->gvs[(g1 * NB + j) * 3 + k];
            s->ang[j][k] = a * M->gavs[(g0 * NB + j) * 3 + k] + b * M->gavs[(g1 * NB + j) * 3 + k];
        }
        q_slerp_f(&M->grs[(g0 * NB + j) * 4], &M->grs[(g1 * NB + j) * 4], b, s->rot[j]);
    }
    if (want_dof) {
        for (int j = 1; j < NB; ++j) {
            R lr[4];
            q_slerp_f(&M->lrs[(g0 * NB + j) * 4], &M->lrs[(g1 * NB + j) * 4], b, lr);
            q_to_exp_map(lr, &s->dof_pos[(j - 1) * 3]);
            for (int k = 0; k < 3; ++k)
                s->dof_vel[(j - 1) * 3 + k] = a * M->dvs[(g0 * (NB - 1) + j - 1) * 3 + k] + b * M->dvs[(g1 * (NB - 1) + j - 1) * 3 + k];
        }
    }
}

void ho_motion_state(const ho_motion* M, int k, const int64_t* ids, const float* times, const float* offset,
                     float* rg_pos, float* rb_rot, float* body_vel, float* body_ang_vel, float* dof_pos, float* dof_vel) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < k; ++i) {
        mstate s;
        motion_eval(M, ids[i], times[i], offset ? offset + 3 * i : NULL, 1, &s);
        for (int j = 0; j < NB; ++j) {
            for (int c = 0; c < 3; ++c) {
                rg_pos[(i * NB + j) * 3 + c] = (float)s.pos[j][c];
                body_vel[(i * NB + j) * 3 + c] = (float)s.vel[j][c];
                body_ang_vel[(i * NB + j) * 3 + c] = (float)s.ang[j][c];
            }
            for (int c = 0; c < 4; ++c) rb_rot[(i * NB + j) * 4 + c] = (float)s.rot[j][c];
        }
        for (int d = 0; d < ND; ++d) { dof_pos[i * ND + d] = (float)s.dof_pos[d]; dof_vel[i * ND + d] = (float)s.dof_vel[d]; }
    }
}

/* motion_lib.py:526-535 (float32 ops as torch does them) */
float ho_sample_time_interval(float phase, float len) {
    const float curr = (float)(1.0 / 30.0);
    float x = (phase * len) / curr;
    int64_t k = (int64_t)x;
    return (float)k * curr;
}

typedef struct sim_body {
    R pos[NB][3], rot[NB][4], vel[NB][3], ang[NB][3];
} sim_body;

static void load_rb(const float* rb, sim_body* s) { /* rb [24,13] */
    for (int j = 0; j < NB; ++j) {
        const float* r = rb + j * 13;
        for (int c = 0; c < 3; ++c) { s->pos[j][c] = r[c]; s->vel[j][c] = r[7 + c]; s->ang[j][c] = r[10 + c]; }
        for (int c = 0; c < 4; ++c) s->rot[j][c] = r[3 + c];
    }
}

/* common.py:22-103 with local_root_obs=True, root_height_obs=True, upright=True, no shape/limb obs */
static void self_obs(const sim_body* s, float* o) {
    R hinv[4];
    heading_quat(-calc_heading(s->rot[0]), hinv);
    o[0] = (float)s->pos[0][2];
    for (int j = 1; j < NB; ++j) {
        R d[3], r[3];
        v3_sub(s->pos[j], s->pos[0], d);
        q_rot(hinv, d, r);
        for (int c = 0; c < 3; ++c) o[1 + (j - 1) * 3 + c] = (float)r[c];
    }
    for (int j = 0; j < NB; ++j) {
        R q[4], tn[6], r[3];
        q_mul(hinv, s->rot[j], q);
        q_tan_norm(q, tn);
        for (int c = 0; c < 6; ++c) o[70 + j * 6 + c] = (float)tn[c];
        q_rot(hinv, s->vel[j], r);
        for (int c = 0; c < 3; ++c) o[214 + j * 3 + c] = (float)r[c];
        q_rot(hinv, s->ang[j], r);
        for (int c = 0; c < 3; ++c) o[286 + j * 3 + c] = (float)r[c];
    }
}

/* common.py:106-176 compute_imitation_observations_v6, time_steps=1, upright=True */
static void task_obs(const sim_body* s, const mstate* m, float* o) {
    R h = calc_heading(s->rot[0]), hinv[4], hq[4];
    heading_quat(-h, hinv);
    heading_quat(h, hq);
    for (int j = 0; j < NB; ++j) {
        R d[3], r[3], q[4], q2[4], cq[4], tn[6];
        v3_sub(m->pos[j], s->pos[j], d); q_rot(hinv, d, r);
        for (int c = 0; c < 3; ++c) o[j * 3 + c] = (float)r[c];
        q_conj(s->rot[j], cq); q_mul(m->rot[j], cq, q); q_mul(hinv, q, q2); q_mul(q2, hq, q); q_tan_norm(q, tn);
        for (int c = 0; c < 6; ++c) o[72 + j * 6 + c] = (float)tn[c];
        v3_sub(m->vel[j], s->vel[j], d); q_rot(hinv, d, r);
        for (int c = 0; c < 3; ++c) o[216 + j * 3 + c] = (float)r[c];
        v3_sub(m->ang[j], s->ang[j], d); q_rot(hinv, d, r);
        for (int c = 0; c < 3; ++c) o[288 + j * 3 + c] = (float)r[c];
        v3_sub(m->pos[j], s->pos[0], d); q_rot(hinv, d, r);
        for (int c = 0; c < 3; ++c) o[360 + j * 3 + c] = (float)r[c];
        q_mul(hinv, m->rot[j], q); q_tan_norm(q, tn);
        for (int c = 0; c < 6; ++c) o[432 + j * 6 + c] = (float)tn[c];
    }
}

/* float32 env time exactly as the torch glue builds it (humanoid_phc.py:1236-1238, 1063-1067) */
static inline float env_time(int progress, float control_dt, float start, float start_off) {
    float t = (float)progress * control_dt;
    t = t + start;
    t = t + start_off;
    return t;
}

/* imitation step for env i (post-physics half of HumanoidPHC.step) */
static void imitation_env(const he_imitation_params* p, const ho_motion* M, int i, const float* rb_state,
                          const float* dof_vel, const float* dof_force, int16_t* progress, const int64_t* motion_ids,
                          const float* start_times, const float* start_offsets, const float* global_offset,
                          float* obs, float* rew, float* reward_raw, uint8_t* reset, uint8_t* terminate) {
    sim_body s;
    load_rb(rb_state + (size_t)i * NB * 13, &s);
    int prog = progress[i] + 1;                     /* humanoid_phc.py:138 */
    progress[i] = (int16_t)prog;
    int64_t mid = motion_ids[i];
    const float* off = global_offset + 3 * i;
    float t = env_time(prog, p->control_dt, start_times[i], start_offsets[i]);
    mstate m;
    motion_eval(M, mid, t, off, 0, &m);
    /* reward, common.py:270-322 */
    R dp = 0, dr = 0, dv = 0, da = 0;
    for (int j = 0; j < NB; ++j) {
        R d[3], q[4], cq[4];
        v3_sub(m.pos[j], s.pos[j], d); dp += v3_dot(d, d) / 3.0;
        v3_sub(m.vel[j], s.vel[j], d); dv += v3_dot(d, d) / 3.0;
        v3_sub(m.ang[j], s.ang[j], d); da += v3_dot(d, d) / 3.0;
        q_conj(s.rot[j], cq); q_mul(m.rot[j], cq, q);
        R ang = q_angle_axis(q, NULL);
        dr += ang * ang;
    }
    dp /= NB; dr /= NB; dv /= NB; da /= NB;
    R rp = exp(-p->k_pos * dp), rr = exp(-p->k_rot * dr), rv = exp(-p->k_vel * dv), ra = exp(-p->k_ang_vel * da);
    R r = p->w_pos * rp + p->w_rot * rr + p->w_vel * rv + p->w_ang_vel * ra;
    reward_raw[i * 5 + 0] = (float)rp; reward_raw[i * 5 + 1] = (float)rr;
    reward_raw[i * 5 + 2] = (float)rv; reward_raw[i * 5 + 3] = (float)ra;
    reward_raw[i * 5 + 4] = 0.0f;
    if (p->use_power_reward) { /* humanoid_phc.py:1297-1305 */
        R pw = 0;
        for (int d = 0; d < ND; ++d) pw += fabs((R)dof_force[i * ND + d] * (R)dof_vel[i * ND + d]);
        R pr = -p->power_coef * pw;
        if (prog <= 3) pr = 0;
        r += pr;
        reward_raw[i * 5 + 4] = (float)pr;
    }
    rew[i] = (float)r;
    /* reset, common.py:325-364 + humanoid_phc.py:1313-1335 */
    int pass_time = t >= M->lengths[mid];
    int fallen = 0;
    if (p->enable_early_termination) {
        if (p->eval_mode) {
            R sum = 0; int cnt = 0; R td = -1;
            for (int j = 0; j < NB; ++j) if (p->reset_body_mask >> j & 1) {
                R d[3]; v3_sub(s.pos[j], m.pos[j], d); sum += v3_norm(d); ++cnt;
                if (td < 0) td = p->term_dist[j];
            }
            fallen = cnt > 0 && (sum / cnt) > td;
        } else {
            for (int j = 0; j < NB; ++j) if (p->reset_body_mask >> j & 1) {
                R d[3]; v3_sub(s.pos[j], m.pos[j], d);
                if (v3_norm(d) > p->term_dist[j]) fallen = 1;
            }
        }
        fallen = fallen && prog > 1;
    }
    terminate[i] = (uint8_t)fallen;
    reset[i] = (uint8_t)(pass_time ? 1 : fallen);
    /* observations for the next step (humanoid_phc.py:1063-1067: time at progress+1) */
    float t2 = env_time(prog + 1, p->control_dt, start_times[i], start_offsets[i]);
    motion_eval(M, mid, t2, off, 0, &m);
    self_obs(&s, obs + (size_t)i * HE_OBS_DIM);
    task_obs(&s, &m, obs + (size_t)i * HE_OBS_DIM + HE_OBS_SELF);
}

void ho_imitation_step(const he_imitation_params* p, const ho_motion* M, int n, const float* rb_state,
                       const float* dof_vel, const float* dof_force, int16_t* progress, const int64_t* motion_ids,
                       const float* start_times, const float* start_offsets, const float* global_offset, float* obs,
                       float* rew, float* reward_raw, uint8_t* reset, uint8_t* terminate) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; ++i)
        imitation_env(p, M, i, rb_state, dof_vel, dof_force, progress, motion_ids, start_times, start_offsets,
                      global_offset, obs, rew, reward_raw, reset, terminate);
}

/* humanoid_phc.py:694-731 + 747-780 + 901-931 + obs for the reset envs */
/* The state init of a reset from its uniform draw u (include/humanoid_engine.h, the StateInit
 * block): 1 = a reference-state init at phase *ph (humanoid_phc.py:694-731, 848-856), 0 = the
 * initial pose (_reset_default, :688-692); Hybrid = Bernoulli(hybrid_init_prob) of the two
 * (:733-745), its phase u / p uniform given the draw. float32 as the kernels. */
static int resolve_init(const he_imitation_params* p, float u, float* ph) {
    int ref = p->state_init != HE_STATE_INIT_DEFAULT;
    *ph = u;
    if (p->state_init == HE_STATE_INIT_HYBRID) {
        ref = u < p->hybrid_init_prob;
        *ph = ref ? u / p->hybrid_init_prob : 0.0f;
    }
    if (p->state_init == HE_STATE_INIT_START || p->test_mode) *ph = 0.0f;
    return ref;
}

/* _reset_default + _reset_env_tensors (humanoid_phc.py:688-692, 747-780): the initial root state,
 * zero dof state and targets, the zero pose's rigid-body rows (every local rotation the identity:
 * body origin = root + R_root rest[b], the root's rotation and velocities), zero contact forces,
 * progress 0; the motion bookkeeping is left as it is (the reference does not touch it). */
static void default_reset(const he_imitation_params* p, const ho_motion* M, int e, const int64_t* motion_ids,
                          const float* start_times, const float* start_offsets, const float* global_offset,
                          int16_t* progress, float* root_states, float* dof_state, float* dof_targets, float* rb_state,
                          float* contact_forces, float* obs, uint8_t* reset, uint8_t* terminate, const float* init_root,
                          const float* rest_pos) {
    const float* ir = init_root + (size_t)e * 13;
    float* rs = root_states + (size_t)e * 13;
    for (int c = 0; c < 13; ++c) rs[c] = ir[c];
    for (int d = 0; d < ND; ++d) {
        dof_state[((size_t)e * ND + d) * 2 + 0] = 0.0f;
        dof_state[((size_t)e * ND + d) * 2 + 1] = 0.0f;
        if (dof_targets) dof_targets[(size_t)e * ND + d] = 0.0f;
    }
    R q[4] = {ir[3], ir[4], ir[5], ir[6]}, w[3] = {ir[10], ir[11], ir[12]};
    float* rb = rb_state + (size_t)e * NB * 13;
    for (int j = 0; j < NB; ++j) {
        R lo[3] = {rest_pos[3 * j], rest_pos[3 * j + 1], rest_pos[3 * j + 2]}, ro[3], wx[3];
        q_rot(q, lo, ro);
        v3_cross(w, ro, wx);
        for (int c = 0; c < 3; ++c) {
            rb[j * 13 + c] = (float)(ir[c] + ro[c]);
            rb[j * 13 + 7 + c] = (float)(ir[7 + c] + wx[c]);
            rb[j * 13 + 10 + c] = ir[10 + c];
        }
        for (int c = 0; c < 4; ++c) rb[j * 13 + 3 + c] = ir[3 + c];
        if (contact_forces) for (int c = 0; c < 3; ++c) contact_forces[((size_t)e * NB + j) * 3 + c] = 0.0f;
    }
    progress[e] = 0;
    if (reset) reset[e] = 0;
    if (terminate) terminate[e] = 0;
    if (obs) {  /* the observation against the env's (unchanged) motion at t(progress 1) */
        int64_t mid = motion_ids[e];
        sim_body s;
        load_rb(rb, &s);
        float t2 = env_time(1, p->control_dt, start_times[e], start_offsets[e]);
        mstate m2;
        motion_eval(M, mid, t2, global_offset + 3 * e, 0, &m2);
        self_obs(&s, obs + (size_t)e * HE_OBS_DIM);
        task_obs(&s, &m2, obs + (size_t)e * HE_OBS_DIM + HE_OBS_SELF);
    }
}

static void reset_env(const he_imitation_params* p, const ho_motion* M, int e, float u, const int64_t* motion_ids,
                      float* start_times, float* start_offsets, float* global_offset, int16_t* progress,
                      float* root_states, float* dof_state, float* dof_targets, float* rb_state, float* contact_forces,
                      float* obs, uint8_t* reset, uint8_t* terminate, const float* init_root, const float* rest_pos) {
    float phase;
    if (!resolve_init(p, u, &phase)) {
        default_reset(p, M, e, motion_ids, start_times, start_offsets, global_offset, progress, root_states, dof_state,
                      dof_targets, rb_state, contact_forces, obs, reset, terminate, init_root, rest_pos);
        return;
    }
    int64_t mid = motion_ids[e];
    float t = ho_sample_time_interval(phase, M->lengths[mid]);
    mstate m;
    motion_eval(M, mid, t, global_offset + 3 * e, 1, &m); /* uses the pre-reset offset (:858-860) */
    float* rs = root_states + (size_t)e * 13;
    for (int c = 0; c < 3; ++c) { rs[c] = (float)m.pos[0][c]; rs[7 + c] = (float)m.vel[0][c]; rs[10 + c] = (float)m.ang[0][c]; }
    for (int c = 0; c < 4; ++c) rs[3 + c] = (float)m.rot[0][c];
    for (int d = 0; d < ND; ++d) {
        dof_state[((size_t)e * ND + d) * 2 + 0] = (float)m.dof_pos[d];
        dof_state[((size_t)e * ND + d) * 2 + 1] = (float)m.dof_vel[d];
        if (dof_targets) dof_targets[(size_t)e * ND + d] = (float)m.dof_pos[d];
    }
    float* rb = rb_state + (size_t)e * NB * 13;
    for (int j = 0; j < NB; ++j) {
        for (int c = 0; c < 3; ++c) { rb[j * 13 + c] = (float)m.pos[j][c]; rb[j * 13 + 7 + c] = (float)m.vel[j][c]; rb[j * 13 + 10 + c] = (float)m.ang[j][c]; }
        for (int c = 0; c < 4; ++c) rb[j * 13 + 3 + c] = (float)m.rot[j][c];
        if (contact_forces) for (int c = 0; c < 3; ++c) contact_forces[((size_t)e * NB + j) * 3 + c] = 0.0f;
    }
    global_offset[3 * e] = global_offset[3 * e + 1] = global_offset[3 * e + 2] = 0.0f;
    start_times[e] = t;
    start_offsets[e] = 0.0f;
    progress[e] = 0;
    if (reset) reset[e] = 0;
    if (terminate) terminate[e] = 0;
    if (obs) {
        sim_body s;
        load_rb(rb, &s);
        float t2 = env_time(1, p->control_dt, t, 0.0f);
        mstate m2;
        motion_eval(M, mid, t2, global_offset + 3 * e, 0, &m2);
        self_obs(&s, obs + (size_t)e * HE_OBS_DIM);
        task_obs(&s, &m2, obs + (size_t)e * HE_OBS_DIM + HE_OBS_SELF);
    }
}

void ho_reset_envs(const he_imitation_params* p, const ho_motion* M, int k, const int32_t* env_ids, const float* phases,
                   const int64_t* motion_ids, float* start_times, float* start_offsets, float* global_offset,
                   int16_t* progress, float* root_states, float* dof_state, float* dof_targets, float* rb_state,
                   float* contact_forces, float* obs, uint8_t* reset, uint8_t* terminate, const float* init_root,
                   const float* rest_pos) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < k; ++i)
        reset_env(p, M, env_ids[i], phases[i], motion_ids, start_times, start_offsets, global_offset, progress,
                  root_states, dof_state, dof_targets, rb_state, contact_forces, obs, reset, terminate, init_root,
                  rest_pos);
}

/* counter-based uniform in [0,1) shared by engine and oracle (splitmix64 finaliser) */
float ho_hash_uniform(uint64_t seed, uint64_t step, uint32_t env) {
    uint64_t z = seed * 0x9E3779B97F4A7C15ull ^ (step + 0x632BE59BD9B4E019ull) * 0xBF58476D1CE4E5B9ull ^
                 ((uint64_t)env + 0x2545F4914F6CDD1Dull) * 0x94D049BB133111EBull;
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)(z >> 40) * (1.0f / 16777216.0f);
}

/* Function-level entry for the golden tests: common.py reward / reset / obs on explicit sim and
 * reference body states (no motion sampling). Arrays [N,24,3|4]; reset uses pass_time[N] and
 * progress[N] as given (already incremented). */
void ho_imitation_from_ref(const he_imitation_params* p, int n, const float* pos, const float* rot, const float* vel,
                           const float* ang, const float* rpos, const float* rrot, const float* rvel, const float* rang,
                           const int16_t* progress, const uint8_t* pass_time, float* rew, float* raw, uint8_t* reset,
                           uint8_t* terminate, float* obs_self, float* obs_task) {
    for (int i = 0; i < n; ++i) {
        sim_body s;
        mstate m;
        for (int j = 0; j < NB; ++j) {
            size_t b3 = ((size_t)i * NB + j) * 3, b4 = ((size_t)i * NB + j) * 4;
            for (int c = 0; c < 3; ++c) {
                s.pos[j][c] = pos[b3 + c]; s.vel[j][c] = vel[b3 + c]; s.ang[j][c] = ang[b3 + c];
                m.pos[j][c] = rpos[b3 + c]; m.vel[j][c] = rvel[b3 + c]; m.ang[j][c] = rang[b3 + c];
            }
            for (int c = 0; c < 4; ++c) { s.rot[j][c] = rot[b4 + c]; m.rot[j][c] = rrot[b4 + c]; }
        }
        R dp = 0, dr = 0, dv = 0, da = 0;
        for (int j = 0; j < NB; ++j) {
            R d[3], q[4], cq[4];
            v3_sub(m.pos[j], s.pos[j], d); dp += v3_dot(d, d) / 3.0;
            v3_sub(m.vel[j], s.vel[j], d); dv += v3_dot(d, d) / 3.0;
            v3_sub(m.ang[j], s.ang[j], d); da += v3_dot(d, d) / 3.0;
            q_conj(s.rot[j], cq); q_mul(m.rot[j], cq, q);
            R a = q_angle_axis(q, NULL);
            dr += a * a;
        }
        dp /= NB; dr /= NB; dv /= NB; da /= NB;
        R r4[4] = {exp(-p->k_pos * dp), exp(-p->k_rot * dr), exp(-p->k_vel * dv), exp(-p->k_ang_vel * da)};
        rew[i] = (float)(p->w_pos * r4[0] + p->w_rot * r4[1] + p->w_vel * r4[2] + p->w_ang_vel * r4[3]);
        for (int c = 0; c < 4; ++c) raw[i * 4 + c] = (float)r4[c];
        int fallen = 0;
        if (p->eval_mode) {
            R sum = 0; int cnt = 0; R td = -1;
            for (int j = 0; j < NB; ++j) if (p->reset_body_mask >> j & 1) {
                R d[3]; v3_sub(s.pos[j], m.pos[j], d); sum += v3_norm(d); ++cnt; if (td < 0) td = p->term_dist[j];
            }
            fallen = cnt > 0 && sum / cnt > td;
        } else {
            for (int j = 0; j < NB; ++j) if (p->reset_body_mask >> j & 1) {
                R d[3]; v3_sub(s.pos[j], m.pos[j], d); if (v3_norm(d) > p->term_dist[j]) fallen = 1;
            }
        }
        fallen = p->enable_early_termination && fallen && progress[i] > 1;
        terminate[i] = (uint8_t)fallen;
        reset[i] = (uint8_t)(pass_time[i] ? 1 : fallen);
        self_obs(&s, obs_self + (size_t)i * HE_OBS_SELF);
        task_obs(&s, &m, obs_task + (size_t)i * HE_OBS_TASK);
    }
}

/* ------------------------------------------------------------------------------------- */
/* AMP observations                                                          */
/* ------------------------------------------------------------------------------------- */
/* common.py:191-267 build_amp_observations_smpl with the constant flags humanoid_phc.py:1195-1210
 * passes (local_root_obs, amp_root_height_obs, has_dof_subset and has_upright_start true; no shape
 * or limb-weight obs), and dof_to_obs_smpl common.py:179-188. The dof subset is given as joint
 * indices (humanoid_phc.py:186-194: the joints outside REMOVE_NAMES). One row per env:
 * [root_h, tan_norm(h^-1 q_root) 6, h^-1 v_root 3, h^-1 w_root 3, tan_norm(exp(dof_j)) 6*J,
 *  dof_vel 3*J, h^-1 (p_key - p_root) 3*K], K = 4 key bodies (body_sets.py:45). */
void ho_amp_obs(int n, int num_joints, const int32_t* joints, int num_key, const float* root_pos,
                const float* root_rot, const float* root_vel, const float* root_ang_vel, const float* dof_pos,
                const float* dof_vel, const float* key_pos, float* out) {
    const int width = 13 + 9 * num_joints + 3 * num_key;
    for (int i = 0; i < n; ++i) {
        R rp[3], rq[4], rv[3], ra[3], hinv[4], q[4], tn[6], r[3];
        for (int c = 0; c < 3; ++c) { rp[c] = root_pos[3 * i + c]; rv[c] = root_vel[3 * i + c]; ra[c] = root_ang_vel[3 * i + c]; }
        for (int c = 0; c < 4; ++c) rq[c] = root_rot[4 * i + c];
        heading_quat(-calc_heading(rq), hinv);
        float* o = out + (size_t)i * width;
        o[0] = (float)rp[2];
        q_mul(hinv, rq, q); q_tan_norm(q, tn);
        for (int c = 0; c < 6; ++c) o[1 + c] = (float)tn[c];
        q_rot(hinv, rv, r); for (int c = 0; c < 3; ++c) o[7 + c] = (float)r[c];
        q_rot(hinv, ra, r); for (int c = 0; c < 3; ++c) o[10 + c] = (float)r[c];
        for (int s = 0; s < num_joints; ++s) {
            const int j = joints[s];
            R e[3] = {dof_pos[(size_t)i * ND + 3 * j], dof_pos[(size_t)i * ND + 3 * j + 1], dof_pos[(size_t)i * ND + 3 * j + 2]};
            exp_map_to_q(e, q); q_tan_norm(q, tn);
            for (int c = 0; c < 6; ++c) o[13 + 6 * s + c] = (float)tn[c];
            for (int c = 0; c < 3; ++c) o[13 + 6 * num_joints + 3 * s + c] = dof_vel[(size_t)i * ND + 3 * j + c];
        }
        for (int k = 0; k < num_key; ++k) {
            R d[3];
            for (int c = 0; c < 3; ++c) d[c] = (R)key_pos[((size_t)i * num_key + k) * 3 + c] - rp[c];
            q_rot(hinv, d, r);
            for (int c = 0; c < 3; ++c) o[13 + 9 * num_joints + 3 * k + c] = (float)r[c];
        }
    }
}

/* OpenMP thread count of the oracle's parallel loops (bench.py cpu_baseline: the cores the host
 * grants this process) */
#include <omp.h>
void ho_set_threads(int n) { if (n > 0) omp_set_num_threads(n); }
int ho_get_threads(void) { return omp_get_max_threads(); }
