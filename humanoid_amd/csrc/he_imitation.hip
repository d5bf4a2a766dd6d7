// he_imitation.hip -- fused motion-sampling + imitation reward / reset / observation kernels for
// gfx950. Compiled with -ffp-contract=off: the env time and frame-index
// arithmetic must reproduce the reference's float32 torch ops exactly
// (humanoid_phc.py:1236-1238, motion_lib.py:655-665).
//
// Mapping: one 32-lane group per env (two envs per wave64), lane b = body b (24 of 32 lanes
// active). Per-env reductions (reward means, power, termination) are xor-shuffles inside the
// group; the root pose is broadcast from lane 0. Every env's rigid-body rows (24 x 13 floats) and
// motion frame records (24 x 13 floats, same layout) are read as one contiguous 1248-B span per
// group; observation blocks are written as contiguous 12/24-B-per-lane runs.
#include <hip/hip_runtime.h>

#include "../../include/humanoid_engine.h"
#include "he_kernels.h"
#include "he_math.h"

namespace {

constexpr int NB = HE_NUM_BODIES;
constexpr int ND = HE_NUM_DOF;
constexpr int GROUP = 32;
constexpr int HOT = HE_MOTION_HOT;    // floats per body in a hot frame record
constexpr int COLD = HE_MOTION_COLD;  // floats per body in a cold frame record

#include "he_imitation_env.h"

// ---------------- eval-mode recording (include/humanoid_engine.h he_eval_buffers)
HE_DEV double group_sum_d(double v) {
#pragma unroll
    for (int o = GROUP / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, GROUP);
    return v;
}

// Largest eigenpair of a symmetric 4x4 by cyclic Jacobi (fp64, fully unrolled: register-resident)
template <int P, int Q>
HE_DEV void jacobi_rot(double (&A)[4][4], double (&V)[4][4]) {
    const double apq = A[P][Q];
    if (fabs(apq) < 1e-300) return;
    const double th = (A[Q][Q] - A[P][P]) / (2.0 * apq);
    const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
    const double c = 1.0 / sqrt(t * t + 1.0), sn = t * c;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double akp = A[k][P], akq = A[k][Q];
        A[k][P] = c * akp - sn * akq;
        A[k][Q] = sn * akp + c * akq;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double apk = A[P][k], aqk = A[Q][k];
        A[P][k] = c * apk - sn * aqk;
        A[Q][k] = sn * apk + c * aqk;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const double vkp = V[k][P], vkq = V[k][Q];
        V[k][P] = c * vkp - sn * vkq;
        V[k][Q] = sn * vkp + c * vkq;
    }
}

// p_mpjpe (smpl_sim smpl_eval, the VideoPose3D "protocol #2"): per-joint error after the
// similarity transform (scale, rotation, translation) that best maps pred onto target. The
// reference solves it by a 3x3 SVD with a reflection fix; the same optimum is the top eigenpair of
// Horn's 4x4 quaternion matrix (eigenvalue = trace of the sign-fixed singular values), used here.
// Lanes = joints; y = pred, x = target (both root-relative), fp64 inside.
HE_DEV float pa_mpjpe_group(bool act, f3 yf, f3 xf) {
    const double yx = act ? yf.x : 0.0, yy = act ? yf.y : 0.0, yz = act ? yf.z : 0.0;
    const double xx = act ? xf.x : 0.0, xy = act ? xf.y : 0.0, xz = act ? xf.z : 0.0;
    const double my[3] = {group_sum_d(yx) / NB, group_sum_d(yy) / NB, group_sum_d(yz) / NB};
    const double mx[3] = {group_sum_d(xx) / NB, group_sum_d(xy) / NB, group_sum_d(xz) / NB};
    const double Y[3] = {act ? yx - my[0] : 0.0, act ? yy - my[1] : 0.0, act ? yz - my[2] : 0.0};
    const double X[3] = {act ? xx - mx[0] : 0.0, act ? xy - mx[1] : 0.0, act ? xz - mx[2] : 0.0};
    double S[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) S[i][j] = group_sum_d(Y[i] * X[j]);
    const double yn = group_sum_d(Y[0] * Y[0] + Y[1] * Y[1] + Y[2] * Y[2]);
    double A[4][4] = {{S[0][0] + S[1][1] + S[2][2], S[1][2] - S[2][1], S[2][0] - S[0][2], S[0][1] - S[1][0]},
                      {S[1][2] - S[2][1], S[0][0] - S[1][1] - S[2][2], S[0][1] + S[1][0], S[2][0] + S[0][2]},
                      {S[2][0] - S[0][2], S[0][1] + S[1][0], -S[0][0] + S[1][1] - S[2][2], S[1][2] + S[2][1]},
                      {S[0][1] - S[1][0], S[2][0] + S[0][2], S[1][2] + S[2][1], -S[0][0] - S[1][1] + S[2][2]}};
    double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
#pragma unroll 1
    for (int sweep = 0; sweep < 10; ++sweep) {
        jacobi_rot<0, 1>(A, V); jacobi_rot<0, 2>(A, V); jacobi_rot<0, 3>(A, V);
        jacobi_rot<1, 2>(A, V); jacobi_rot<1, 3>(A, V); jacobi_rot<2, 3>(A, V);
        const double off = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[0][3] * A[0][3] + A[1][2] * A[1][2] +
                           A[1][3] * A[1][3] + A[2][3] * A[2][3];
        const double dia = A[0][0] * A[0][0] + A[1][1] * A[1][1] + A[2][2] * A[2][2] + A[3][3] * A[3][3];
        if (off <= 1e-30 * dia) break;  // converged to fp64 rounding (typically 3-4 sweeps)
    }
    int k = 0;
    double lam = A[0][0];
#pragma unroll
    for (int i = 1; i < 4; ++i)
        if (A[i][i] > lam) { lam = A[i][i]; k = i; }
    double q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = k == 0 ? V[i][0] : (k == 1 ? V[i][1] : (k == 2 ? V[i][2] : V[i][3]));
    const double qn = 1.0 / sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    const double w = q[0] * qn, vx = q[1] * qn, vy = q[2] * qn, vz = q[3] * qn;
    const double scale = lam / yn;
    // Q y = y + 2w (v x y) + 2 v x (v x y)
    const double c1x = vy * Y[2] - vz * Y[1], c1y = vz * Y[0] - vx * Y[2], c1z = vx * Y[1] - vy * Y[0];
    const double c2x = vy * c1z - vz * c1y, c2y = vz * c1x - vx * c1z, c2z = vx * c1y - vy * c1x;
    const double ex = scale * (Y[0] + 2.0 * (w * c1x + c2x)) - X[0];
    const double ey = scale * (Y[1] + 2.0 * (w * c1y + c2y)) - X[1];
    const double ez = scale * (Y[2] + 2.0 * (w * c1z + c2z)) - X[2];
    const double err = act ? sqrt(ex * ex + ey * ey + ez * ez) : 0.0;
    return (float)(group_sum_d(err) / NB);
}

// One eval frame of env e (lane b = body): p = simulated body position, g = reference rg_pos.
HE_DEV void eval_record(const he_eval_buffers& ev, int e, int lane, bool act, f3 p, f3 g) {
    const int b = act ? lane : 0;
    const int s = ev.frame;
    // extras["mpjpe"] = (body_pos - rg_pos).norm(dim=-1).mean(dim=-1) (humanoid_phc.py:165)
    const float dist = act ? norm3(p - g) : 0.0f;
    const float mp = group_sum(dist) / NB;
    if (lane == 0 && ev.mpjpe) ev.mpjpe[e] = mp;
    if (act && ev.body_pos) { float* o = ev.body_pos + ((size_t)e * NB + b) * 3; o[0] = p.x; o[1] = p.y; o[2] = p.z; }
    if (act && ev.body_pos_gt) { float* o = ev.body_pos_gt + ((size_t)e * NB + b) * 3; o[0] = g.x; o[1] = g.y; o[2] = g.z; }
    double* sum = ev.sums + (size_t)e * HE_EVAL_SUMS;
    float* hist = ev.history + (size_t)e * (2 * 2 * NB * 3);  // [slot][pred, gt][NB][3]
    auto H = [&](int slot, int which) { return hist + ((slot * 2 + which) * NB + b) * 3; };
    if (s == 0 && lane == 0)
        for (int k = 0; k < HE_EVAL_SUMS; ++k) sum[k] = 0.0;
    if (s < ev.num_steps[e] - 1) {  // the frame is inside the [: (i - 1)] slice (phc_train.py:146-151)
        // compute_metrics_lite per frame (x 1000 = mm): mpjpe_g on world positions ...
        const float mg = group_sum(act ? norm3(g - p) : 0.0f) / NB * 1000.0f;
        // ... mpjpe_l and p_mpjpe on root-relative positions
        const f3 p0 = f3{__shfl(p.x, 0, GROUP), __shfl(p.y, 0, GROUP), __shfl(p.z, 0, GROUP)};
        const f3 g0 = f3{__shfl(g.x, 0, GROUP), __shfl(g.y, 0, GROUP), __shfl(g.z, 0, GROUP)};
        const f3 pr = p - p0, gr = g - g0;
        const float ml = group_sum(act ? norm3(pr - gr) : 0.0f) / NB * 1000.0f;
        const float pa = pa_mpjpe_group(act, pr, gr) * 1000.0f;
        float vel = 0.0f, acc = 0.0f;
        if (s >= 1) {  // compute_error_vel: frame differences
            const float* p1 = H((s - 1) & 1, 0);
            const float* g1 = H((s - 1) & 1, 1);
            const f3 vp = p - f3{p1[0], p1[1], p1[2]}, vg = g - f3{g1[0], g1[1], g1[2]};
            vel = group_sum(act ? norm3(vp - vg) : 0.0f) / NB * 1000.0f;
            if (s >= 2) {  // compute_error_accel: x[t-2] - 2 x[t-1] + x[t]
                const float* p2 = H(s & 1, 0);
                const float* g2 = H(s & 1, 1);
                const f3 ap = (f3{p2[0], p2[1], p2[2]} - f3{p1[0], p1[1], p1[2]} * 2.0f) + p;
                const f3 ag = (f3{g2[0], g2[1], g2[2]} - f3{g1[0], g1[1], g1[2]} * 2.0f) + g;
                acc = group_sum(act ? norm3(ap - ag) : 0.0f) / NB * 1000.0f;
            }
        }
        if (lane == 0) {
            sum[0] += mg; sum[1] += ml; sum[2] += pa;
            sum[5] += 1.0;
            if (s >= 1) { sum[3] += vel; sum[6] += 1.0; }
            if (s >= 2) { sum[4] += acc; sum[7] += 1.0; }
        }
    }
    if (act) {  // this frame becomes history (slot s & 1 held frame s - 2, already read above)
        float* hp = H(s & 1, 0);
        float* hg = H(s & 1, 1);
        hp[0] = p.x; hp[1] = p.y; hp[2] = p.z;
        hg[0] = g.x; hg[1] = g.y; hg[2] = g.z;
    }
}

// EVAL: eval recording compiled in (its fp64 Procrustes solve would otherwise set the register
// budget of every launch)
#ifndef HE_IMIT_THREADS  // threads per workgroup of the imitation kernel
#define HE_IMIT_THREADS 256
#endif
#ifndef HE_IMIT_MIN_WAVES  // waves per SIMD the register budget must allow (launch bound)
#define HE_IMIT_MIN_WAVES 1
#endif
template <bool EVAL>
__global__ void __launch_bounds__(HE_IMIT_THREADS, HE_IMIT_MIN_WAVES) imitation_kernel(ImitArgs a) {
    const int lane = threadIdx.x & (GROUP - 1);
    const int slot = (blockIdx.x * blockDim.x + threadIdx.x) / GROUP;
    if (slot >= a.count) return;  // whole 32-lane group leaves together
    const int e = a.env_ids ? a.env_ids[slot] : slot;
    const bool act = lane < NB;
    const int b = act ? lane : 0;
    const he_imitation_params& p = a.p;
    // Dependent global round trips are the cost of this kernel, so every load that does not depend
    // on a motion-table index is issued first, and both motion samples (t for reward/reset, t+dt
    // for the observation) are selected from one metadata read and loaded together before any store.
    // trip 1: env bookkeeping, the env's motion-metadata cache, the simulated body row, the
    // power-reward operands
    const int64_t mid = clamp_mid(a.m, a.motion_ids[e]);
    int4 mc0 = make_int4(-1, -1, 0, 0), mc1 = make_int4(0, 0, 0, 0);
    if (a.meta_cache) {
        const int4* mc = reinterpret_cast<const int4*>(a.meta_cache + (size_t)e * 8);
        mc0 = mc[0];
        mc1 = mc[1];
    }
    f3 off = f3{a.global_offset[3 * e], a.global_offset[3 * e + 1], a.global_offset[3 * e + 2]};
    float start = a.start_times[e], soff = a.start_offsets[e];
    int prog = a.progress[e];
    SimBody s = load_body(a.rb_state + ((size_t)e * NB + b) * 13);
    float pw = 0.0f;
    if (a.mode != 2 && p.use_power_reward && lane < NB - 1) {  // humanoid_phc.py:1297-1305
        const float* f = a.dof_force + (size_t)e * ND + 3 * lane;
        const float* v = a.dof_state + ((size_t)e * ND + 3 * lane) * 2 + 1;
        pw = power_term(f, v, 2);
    }
    // trip 2 (only when the env's motion changed since its last step, or the tables were reloaded:
    // the cache is keyed by the motion id and cleared on a load): the motion's metadata
    auto i64 = [](int lo, int hi) { return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo); };
    MotionMeta mm;
    if (a.meta_cache && i64(mc0.x, mc0.y) == mid) {  // uniform in the env's group
        mm = MotionMeta{__int_as_float(mc0.z), __int_as_float(mc0.w), i64(mc1.x, mc1.y), i64(mc1.z, mc1.w)};
    } else {
        mm = motion_meta(a.m, mid);
        if (a.meta_cache && lane == 0) {
            int4* mc = reinterpret_cast<int4*>(a.meta_cache + (size_t)e * 8);
            mc[0] = make_int4((int)(uint32_t)mid, (int)((uint64_t)mid >> 32), __float_as_int(mm.len), __float_as_int(mm.dt));
            mc[1] = make_int4((int)(uint32_t)mm.nf, (int)((uint64_t)mm.nf >> 32), (int)(uint32_t)mm.start,
                              (int)((uint64_t)mm.start >> 32));
        }
    }
    imitation_finish<EVAL>(a, slot, e, lane, lane == 0,
                           imitation_frames(a, lane, ImitBook{mid, off, start, soff, prog, mm}), s, pw);
}

// MotionLibBase.get_motion_state for K queries (motion_lib.py:549-626)
__global__ void __launch_bounds__(256) motion_state_kernel(MotionStateArgs a) {
    const int lane = threadIdx.x & (GROUP - 1);
    const int q = (blockIdx.x * blockDim.x + threadIdx.x) / GROUP;
    if (q >= a.k || lane >= NB) return;
    const int b = lane;
    f3 off = a.offset ? f3{a.offset[3 * q], a.offset[3 * q + 1], a.offset[3 * q + 2]} : f3{0.f, 0.f, 0.f};
    FrameSel fs = frame_select(a.m, a.ids[q], a.times[q]);  // clamps the id
    BodyRef r = body_ref(a.m, fs, b, off);
    size_t o3 = ((size_t)q * NB + b) * 3, o4 = ((size_t)q * NB + b) * 4;
    if (a.rg_pos) { a.rg_pos[o3] = r.pos.x; a.rg_pos[o3 + 1] = r.pos.y; a.rg_pos[o3 + 2] = r.pos.z; }
    if (a.rb_rot) { a.rb_rot[o4] = r.rot.x; a.rb_rot[o4 + 1] = r.rot.y; a.rb_rot[o4 + 2] = r.rot.z; a.rb_rot[o4 + 3] = r.rot.w; }
    if (a.body_vel) { a.body_vel[o3] = r.vel.x; a.body_vel[o3 + 1] = r.vel.y; a.body_vel[o3 + 2] = r.vel.z; }
    if (a.body_ang_vel) { a.body_ang_vel[o3] = r.ang.x; a.body_ang_vel[o3 + 1] = r.ang.y; a.body_ang_vel[o3 + 2] = r.ang.z; }
    if (b > 0 && (a.dof_pos || a.dof_vel)) {
        f3 dp, dv;
        body_dof_ref(a.m, fs, b, dp, dv);
        size_t od = (size_t)q * ND + 3 * (b - 1);
        if (a.dof_pos) { a.dof_pos[od] = dp.x; a.dof_pos[od + 1] = dp.y; a.dof_pos[od + 2] = dp.z; }
        if (a.dof_vel) { a.dof_vel[od] = dv.x; a.dof_vel[od + 1] = dv.y; a.dof_vel[od + 2] = dv.z; }
    }
}


// ---------------- AMP observations ---------------------------------------------
// Per body: the AMP dof-subset slot of its joint (humanoid_phc.py:186-194: joints outside
// REMOVE_NAMES, in DOF_NAMES order) and its key-body slot (KEY_BODIES, body_sets.py:45).
__constant__ int8_t kAmpSub[NB] = {-1, 0, 1, 2, -1, 3, 4, 5, -1, 6, 7, 8, 9, 10, 11, 12, 13, 14, -1, 15, 16, 17, 18, -1};
__constant__ int8_t kAmpKey[NB] = {-1, -1, -1, 1, -1, -1, -1, 0, -1, -1, -1, -1, -1, -1, -1, -1, -1, 3, -1, -1, -1, -1, 2, -1};
constexpr int AMP_W = HE_AMP_OBS_STEP;
constexpr int AMP_J = 19;  // kept joints
static_assert(13 + 9 * AMP_J + 3 * 4 == AMP_W, "AMP row layout");

// build_amp_observations_smpl (common.py:191-267) for one row; lane b holds body b's position
// (read on the root and key lanes), the root lane its rotation and velocities, lane b >= 1 its
// joint's exp map and dof velocity. Writes to o (and o2 when non-null).
HE_DEV void amp_row(float* o, float* o2, int lane, bool act, f3 pos, f4 rot, f3 vel, f3 ang, f3 dpos, f3 dvel) {
    const f3 rp = f3{bcast0(pos.x), bcast0(pos.y), bcast0(pos.z)};
    const f4 rq = f4{bcast0(rot.x), bcast0(rot.y), bcast0(rot.z), bcast0(rot.w)};
    const f4 hinv = heading_quat(-calc_heading(rq));  // calc_heading_quat_inv, upright start
    float v[13];
    int n = 0, at = 0;
    if (lane == 0) {
        float tn[6];
        tan_norm(qmul_ref(hinv, rq), tn);  // local_root_obs
        const f3 lv = qrot_ref(hinv, vel), la = qrot_ref(hinv, ang);
        v[0] = rp.z;
        for (int c = 0; c < 6; ++c) v[1 + c] = tn[c];
        v[7] = lv.x; v[8] = lv.y; v[9] = lv.z; v[10] = la.x; v[11] = la.y; v[12] = la.z;
        n = 13;
    }
    const int sub = act ? kAmpSub[lane] : -1;
    const int key = act ? kAmpKey[lane] : -1;
    if (n) {
        for (int c = 0; c < 13; ++c) { o[at + c] = v[c]; if (o2) o2[at + c] = v[c]; }
    }
    if (sub >= 0) {  // dof_to_obs_smpl (common.py:179-188) and the dof velocity subset
        float tn[6];
        tan_norm(exp_map_to_quat_ref(dpos), tn);
        const int d = 13 + 6 * sub, w = 13 + 6 * AMP_J + 3 * sub;
        for (int c = 0; c < 6; ++c) { o[d + c] = tn[c]; if (o2) o2[d + c] = tn[c]; }
        const float dv[3] = {dvel.x, dvel.y, dvel.z};
        for (int c = 0; c < 3; ++c) { o[w + c] = dv[c]; if (o2) o2[w + c] = dv[c]; }
    }
    if (key >= 0) {  // key-body positions in the heading frame
        const f3 lk = qrot_ref(hinv, pos - rp);
        const int k = 13 + 9 * AMP_J + 3 * key;
        const float kv[3] = {lk.x, lk.y, lk.z};
        for (int c = 0; c < 3; ++c) { o[k + c] = kv[c]; if (o2) o2[k + c] = kv[c]; }
    }
}

// _update_hist_amp_obs shift (humanoid_phc.py:1341-1347) of one env's rows 0..S-2 to 1..S-1 by a
// 32-lane group, as float4 (rows are 784 B). Every load of a chunk precedes its stores; chunks go
// from the top down, and the shift (49 float4) exceeds a chunk (32), so no chunk reads what an
// earlier chunk wrote.
HE_DEV void amp_shift(float* buf, int S, int lane) {
    const int n4 = (S - 1) * (AMP_W / 4);
    float4* p = reinterpret_cast<float4*>(buf);
    constexpr int SH = AMP_W / 4;
    if (n4 <= 16 * GROUP) {  // S <= 11: every value in registers first
        float4 r[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int idx = i * GROUP + lane;
            if (idx < n4) r[i] = p[idx];
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int idx = i * GROUP + lane;
            if (idx < n4) p[idx + SH] = r[i];
        }
    } else {
        for (int base = ((n4 - 1) / GROUP) * GROUP; base >= 0; base -= GROUP) {
            const int idx = base + lane;
            float4 r;
            if (idx < n4) r = p[idx];
            if (idx < n4) p[idx + SH] = r;
        }
    }
}

// One 32-lane group per (env, row): row 0's group does the history shift (envs that continue) and
// writes the current row; for envs reset by the preceding launch, the group of row k >= 1 writes the
// motion row k, so the S-1 motion samples of a reset env run in parallel instead of in series.
__global__ void __launch_bounds__(256) amp_kernel(AmpArgs a) {
    const int lane = threadIdx.x & (GROUP - 1);
    const int S = a.amp.num_steps;
    const int gid = (blockIdx.x * blockDim.x + threadIdx.x) / GROUP;
    const int slot = gid / S, k = gid - slot * S;
    if (slot >= a.count) return;  // whole 32-lane group leaves together
    const int e = a.env_ids ? a.env_ids[slot] : slot;
    const bool init = a.mode == 2 || (a.mode == 1 && a.reset[e]);
    if (k > 0 && !init) return;
    // the reset's state init, from the same draw as the imitation launch's (resolve_init)
    bool ref = true;
    if (init) {
        float ph;
        ref = resolve_init(a.ip, a.mode == 2 ? a.phases[slot] : hash_uniform(a.seed, a.step, (uint32_t)e), ph);
    }
    const bool act = lane < NB;
    const int b = act ? lane : 0;
    float* row = a.amp.amp_obs + ((size_t)e * S + k) * AMP_W;
    float* demo = (init && ref && a.amp.amp_obs_demo) ? a.amp.amp_obs_demo + ((size_t)e * S + k) * AMP_W : nullptr;
    // row 0, and for a Default init every history row (_init_amp_obs_default, humanoid_phc.py:801-803:
    // the history is the current observation; the reference raises "Not tested yet" before it,
    // :794-796, and the engine runs the function it left): from the simulated (or just reset) state
    if (k == 0 || !ref) {
        if (k == 0 && !init && S > 1) amp_shift(row, S, lane);
        // _compute_amp_observations from the simulated (or just reset) state
        const SimBody s = load_body(a.rb_state + ((size_t)e * NB + b) * 13);
        f3 dp = f3{0.f, 0.f, 0.f}, dv = f3{0.f, 0.f, 0.f};
        if (act && b > 0) {
            const float* ds = a.dof_state + ((size_t)e * ND + 3 * (b - 1)) * 2;
            dp = f3{ds[0], ds[2], ds[4]};
            dv = f3{ds[1], ds[3], ds[5]};
        }
        amp_row(row, demo, lane, act, s.pos, s.rot, s.vel, s.ang, dp, dv);
        return;
    }
    // _init_amp_obs_ref: the motion at t - k*dt without offset (humanoid_phc.py:805-838)
    const int64_t mid = clamp_mid(a.m, a.motion_ids[e]);
    const float t = a.start_times[e] + (-a.control_dt) * (float)k;
    const FrameSel fs = frame_select(a.m, mid, t);
    const BodyRef r = body_ref(a.m, fs, b, f3{0.f, 0.f, 0.f});
    f3 mp = f3{0.f, 0.f, 0.f}, mv = f3{0.f, 0.f, 0.f};
    if (act && b > 0) body_dof_ref(a.m, fs, b, mp, mv);
    amp_row(row, demo, lane, act, r.pos, r.rot, r.vel, r.ang, mp, mv);
}

// he_amp_observations: explicit inputs, one 32-lane group per row
__global__ void __launch_bounds__(256) amp_function_kernel(AmpArgs a) {
    const int lane = threadIdx.x & (GROUP - 1);
    const int q = (blockIdx.x * blockDim.x + threadIdx.x) / GROUP;
    if (q >= a.count) return;
    const bool act = lane < NB;
    f3 pos = f3{0.f, 0.f, 0.f}, vel = pos, ang = pos, dp = pos, dv = pos;
    f4 rot = f4{0.f, 0.f, 0.f, 1.f};
    if (lane == 0) {
        pos = f3{a.root_pos[3 * q], a.root_pos[3 * q + 1], a.root_pos[3 * q + 2]};
        rot = f4{a.root_rot[4 * q], a.root_rot[4 * q + 1], a.root_rot[4 * q + 2], a.root_rot[4 * q + 3]};
        vel = f3{a.root_vel[3 * q], a.root_vel[3 * q + 1], a.root_vel[3 * q + 2]};
        ang = f3{a.root_ang_vel[3 * q], a.root_ang_vel[3 * q + 1], a.root_ang_vel[3 * q + 2]};
    } else if (act) {
        const int key = kAmpKey[lane];
        if (key >= 0) {
            const float* kp = a.key_pos + ((size_t)q * 4 + key) * 3;
            pos = f3{kp[0], kp[1], kp[2]};
        }
        const size_t d = (size_t)q * ND + 3 * (lane - 1);
        dp = f3{a.dof_pos[d], a.dof_pos[d + 1], a.dof_pos[d + 2]};
        dv = f3{a.dof_vel[d], a.dof_vel[d + 1], a.dof_vel[d + 2]};
    }
    amp_row(a.out + (size_t)q * AMP_W, nullptr, lane, act, pos, rot, vel, ang, dp, dv);
}
}  // namespace

hipError_t launch_imitation(const ImitArgs& a, hipStream_t stream) {
    if (a.count <= 0) return hipSuccess;
    int threads = HE_IMIT_THREADS;
    int blocks = (a.count * GROUP + threads - 1) / threads;
    if (a.has_eval && a.mode != 2)
        imitation_kernel<true><<<blocks, threads, 0, stream>>>(a);
    else
        imitation_kernel<false><<<blocks, threads, 0, stream>>>(a);
    return hipGetLastError();
}

namespace {
__global__ void warm_tu_kernel() {}
}  // namespace

hipError_t warm_imitation_kernels(hipStream_t stream, int mode) {
    if (mode == 1) {
        warm_tu_kernel<<<1, 64, 0, stream>>>();
        return hipGetLastError();
    }
    ImitArgs ia{};
    imitation_kernel<false><<<1, HE_IMIT_THREADS, 0, stream>>>(ia);
    imitation_kernel<true><<<1, HE_IMIT_THREADS, 0, stream>>>(ia);
    MotionStateArgs ma{};
    motion_state_kernel<<<1, 256, 0, stream>>>(ma);
    AmpArgs aa{};
    aa.amp.num_steps = 1;
    amp_kernel<<<1, 256, 0, stream>>>(aa);
    amp_function_kernel<<<1, 256, 0, stream>>>(aa);
    return hipGetLastError();
}

hipError_t launch_motion_state(const MotionStateArgs& a, hipStream_t stream) {
    if (a.k <= 0) return hipSuccess;
    int threads = 256;
    int blocks = (a.k * GROUP + threads - 1) / threads;
    motion_state_kernel<<<blocks, threads, 0, stream>>>(a);
    return hipGetLastError();
}

hipError_t launch_amp(const AmpArgs& a, hipStream_t stream) {
    if (a.count <= 0) return hipSuccess;
    int threads = 256;
    int blocks = (int)(((int64_t)a.count * a.amp.num_steps * GROUP + threads - 1) / threads);
    amp_kernel<<<blocks, threads, 0, stream>>>(a);
    return hipGetLastError();
}

hipError_t launch_amp_function(const AmpArgs& a, hipStream_t stream) {
    if (a.count <= 0) return hipSuccess;
    int threads = 256;
    int blocks = (a.count * GROUP + threads - 1) / threads;
    amp_function_kernel<<<blocks, threads, 0, stream>>>(a);
    return hipGetLastError();
}
