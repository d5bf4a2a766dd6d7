// he_imitation_env.h -- the per-env imitation step on one 32-lane group,
// shared by the stand-alone imitation kernel (he_imitation.hip, two envs per wave) and the physics
// kernel's fused epilogue (he_physics.hip, he_env_step: one env per wave, lanes 0..31).
//
// Included inside each TU's anonymous namespace after he_kernels.h / he_math.h, with NB, ND, GROUP,
// HOT, COLD defined. Everything here reproduces the reference's float32 torch rounding: the physics
// TU includes it under `#pragma clang fp contract(off)` (the imitation TU is compiled with
// -ffp-contract=off), and the shared he_math.h helpers it calls carry the pragma in their bodies.
// Mapping: lane b = body b (24 of 32 lanes active); per-env reductions are xor-shuffles inside the
// group; the root pose is broadcast from lane 0.

// diagnostics only (tools/build_variant.py --tu he_imitation.hip -DHE_IMIT_DIAG=...): bit 0 drops
// the observation math and stores, bit 1 reads the frame records at fixed indices (no dependent
// round trip), bit 2 drops the reward / termination math, bit 3 the frame blends, bit 4 the angle
// term, bit 5 the termination test, bit 6 the device reset of mode 1, bit 7 keeps the reset code but resets no env, to time the rest
// of the step; the product build has 0
#ifndef HE_IMIT_DIAG
#define HE_IMIT_DIAG 0
#endif

HE_DEV float norm3_im(f3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }

// The 32-lane group reductions and the group broadcast on the VALU (HE_IMIT_DPP): DPP steps inside a
// 16-lane row (quad perms, half-row and row mirrors) and one v_permlane16_swap across the group's two
// rows, instead of five LDS-crossbar ds_bpermute round trips; the broadcast by two v_readlane.
// Every lane of a group must be active (the kernels' groups enter and leave whole).
#ifndef HE_IMIT_DPP
#define HE_IMIT_DPP 1
#endif
#if HE_IMIT_DPP
template <int CTRL>
HE_DEV float im_dpp(float x) { return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, false)); }
// {v of the group's even row, v of its odd row} on every lane: v_permlane16_swap of v with itself
HE_DEV void im_rows(float v, float& r0, float& r1) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    r0 = __uint_as_float(r[0]);
    r1 = __uint_as_float(r[1]);
}
HE_DEV float group_sum(float v) {
    v += im_dpp<0xB1>(v);   // quad_perm [1,0,3,2]
    v += im_dpp<0x4E>(v);   // quad_perm [2,3,0,1]
    v += im_dpp<0x141>(v);  // row_half_mirror: the other quad of the 8
    v += im_dpp<0x140>(v);  // row_mirror: the other 8 of the row
    float r0, r1;
    im_rows(v, r0, r1);     // one of the two is v itself, the other the other row's sum
    return r0 + r1;
}
HE_DEV float group_max(float v) {
    v = fmaxf(v, im_dpp<0xB1>(v));
    v = fmaxf(v, im_dpp<0x4E>(v));
    v = fmaxf(v, im_dpp<0x141>(v));
    v = fmaxf(v, im_dpp<0x140>(v));
    float r0, r1;
    im_rows(v, r0, r1);
    return fmaxf(r0, r1);
}
HE_DEV float bcast0(float v) {
    const float a = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float b = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    return (threadIdx.x & 32) ? b : a;
}
#else
HE_DEV float group_sum(float v) {
#pragma unroll
    for (int o = GROUP / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, GROUP);
    return v;
}
HE_DEV float group_max(float v) {
#pragma unroll
    for (int o = GROUP / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, GROUP));
    return v;
}
HE_DEV float bcast0(float v) { return __shfl(v, 0, GROUP); }
#endif

struct FrameSel {
    int64_t g0, g1;
    float blend;
};

// motion_lib.py:655-665 in float32
HE_DEV int64_t clamp_mid(const MotionDev& m, int64_t mid) {
    return mid < 0 ? 0 : (mid >= m.num_motions ? (int64_t)m.num_motions - 1 : mid);
}

struct MotionMeta {
    float len, dt;
    int64_t nf, start;
};

HE_DEV MotionMeta motion_meta(const MotionDev& m, int64_t mid) {  // mid already clamped
    return MotionMeta{m.lengths[mid], m.dt[mid], m.num_frames[mid], m.length_starts[mid]};
}

HE_DEV FrameSel frame_select(const MotionMeta& mm, float time) {
    const float len = mm.len, dt = mm.dt;
    const int64_t nf = mm.nf;
    float phase = time / len;
    phase = phase < 0.0f ? 0.0f : (phase > 1.0f ? 1.0f : phase);
    if (time < 0.0f) time = 0.0f;
    int64_t f0 = (int64_t)(phase * (float)(nf - 1));
    int64_t f1 = f0 + 1 < nf - 1 ? f0 + 1 : nf - 1;
    float bl = (time - (float)f0 * dt) / dt;
    bl = bl < 0.0f ? 0.0f : (bl > 1.0f ? 1.0f : bl);
    return FrameSel{mm.start + f0, mm.start + f1, bl};
}

HE_DEV FrameSel frame_select(const MotionDev& m, int64_t mid, float time) {
    mid = clamp_mid(m, mid);
    float len = m.lengths[mid];
    int64_t nf = m.num_frames[mid];
    float dt = m.dt[mid];
    float phase = time / len;
    phase = phase < 0.0f ? 0.0f : (phase > 1.0f ? 1.0f : phase);
    if (time < 0.0f) time = 0.0f;
    int64_t f0 = (int64_t)(phase * (float)(nf - 1));
    int64_t f1 = f0 + 1 < nf - 1 ? f0 + 1 : nf - 1;
    float bl = (time - (float)f0 * dt) / dt;
    bl = bl < 0.0f ? 0.0f : (bl > 1.0f ? 1.0f : bl);
    int64_t s = m.length_starts[mid];
    return FrameSel{s + f0, s + f1, bl};
}

struct BodyRef {
    f3 pos, vel, ang;
    f4 rot;
};

// the two frame records of one body's sample, loaded (body_ref_blend does the arithmetic)
struct RefRows {
    float r0[HOT], r1[HOT];
    float blend;
};
HE_DEV RefRows body_ref_load(const MotionDev& m, const FrameSel& fs, int b) {
    RefRows x;
    const float* r0 = m.hot + (fs.g0 * NB + b) * HOT;
    const float* r1 = m.hot + (fs.g1 * NB + b) * HOT;
#pragma unroll
    for (int c = 0; c < HOT; ++c) { x.r0[c] = r0[c]; x.r1[c] = r1[c]; }
    x.blend = fs.blend;
    return x;
}
// motion_lib.py:577-610 for one body
HE_DEV BodyRef body_ref_blend(const RefRows& x, f3 off) {
    const float* r0 = x.r0;
    const float* r1 = x.r1;
    float bl = x.blend, a = 1.0f - bl;
    BodyRef o;
#if HE_IMIT_DIAG & 8  // no blend: the first frame's record
    o.pos = f3{r0[0] + off.x, r0[1] + r1[1], r0[2]};
    o.rot = f4{r0[3], r0[4], r0[5], r0[6] + bl};
    o.vel = f3{r0[7], r0[8], r0[9]};
    o.ang = f3{r0[10], r0[11], r0[12]};
    return o;
#endif
    o.pos = f3{a * r0[0] + bl * r1[0], a * r0[1] + bl * r1[1], a * r0[2] + bl * r1[2]};
    o.pos = o.pos + off;
    o.rot = slerp_ref(f4{r0[3], r0[4], r0[5], r0[6]}, f4{r1[3], r1[4], r1[5], r1[6]}, bl);
    o.vel = f3{a * r0[7] + bl * r1[7], a * r0[8] + bl * r1[8], a * r0[9] + bl * r1[9]};
    o.ang = f3{a * r0[10] + bl * r1[10], a * r0[11] + bl * r1[11], a * r0[12] + bl * r1[12]};
    return o;
}
HE_DEV BodyRef body_ref(const MotionDev& m, const FrameSel& fs, int b, f3 off) {
    return body_ref_blend(body_ref_load(m, fs, b), off);
}

struct ColdRows {
    float c0[COLD], c1[COLD];
    float blend;
};
HE_DEV ColdRows body_cold_load(const MotionDev& m, const FrameSel& fs, int b) {
    ColdRows x;
    const float* c0 = m.cold + (fs.g0 * NB + b) * COLD;
    const float* c1 = m.cold + (fs.g1 * NB + b) * COLD;
#pragma unroll
    for (int c = 0; c < COLD; ++c) { x.c0[c] = c0[c]; x.c1[c] = c1[c]; }
    x.blend = fs.blend;
    return x;
}
// local rotation slerp -> exp-map dof pos, dof vel lerp (motion_lib.py:562-606, 670-673)
HE_DEV void body_dof_blend(const ColdRows& x, f3& dpos, f3& dvel) {
    const float bl = x.blend, a = 1.0f - bl;
    const f4 lr = slerp_ref(f4{x.c0[0], x.c0[1], x.c0[2], x.c0[3]}, f4{x.c1[0], x.c1[1], x.c1[2], x.c1[3]}, bl);
    dpos = q_to_exp_map(lr);
    dvel = f3{a * x.c0[4] + bl * x.c1[4], a * x.c0[5] + bl * x.c1[5], a * x.c0[6] + bl * x.c1[6]};
}
HE_DEV void body_dof_ref(const MotionDev& m, const FrameSel& fs, int b, f3& dpos, f3& dvel) {
    body_dof_blend(body_cold_load(m, fs, b), dpos, dvel);
}

HE_DEV float env_time(int progress, float cdt, float start, float off) {
    float t = (float)progress * cdt;
    t = t + start;
    t = t + off;
    return t;
}

struct SimBody {
    f3 pos, vel, ang;
    f4 rot;
};

HE_DEV SimBody load_body(const float* rb) {
    SimBody s;
    s.pos = f3{rb[0], rb[1], rb[2]};
    s.rot = f4{rb[3], rb[4], rb[5], rb[6]};
    s.vel = f3{rb[7], rb[8], rb[9]};
    s.ang = f3{rb[10], rb[11], rb[12]};
    return s;
}

// common.py:22-103 (self) and :106-176 (task, time_steps=1) for body b of one env
HE_DEV void write_obs(float* o, int b, const SimBody& s, f3 root_pos, f4 hinv, f4 hq, const BodyRef& r) {
    float tn[6];
    if (b == 0) o[0] = root_pos.z;
    if (b > 0) {
        f3 lp = qrot_ref(hinv, s.pos - root_pos);
        o[1 + (b - 1) * 3 + 0] = lp.x; o[1 + (b - 1) * 3 + 1] = lp.y; o[1 + (b - 1) * 3 + 2] = lp.z;
    }
    tan_norm(qmul_ref(hinv, s.rot), tn);
#pragma unroll
    for (int c = 0; c < 6; ++c) o[70 + b * 6 + c] = tn[c];
    f3 v = qrot_ref(hinv, s.vel);
    o[214 + b * 3 + 0] = v.x; o[214 + b * 3 + 1] = v.y; o[214 + b * 3 + 2] = v.z;
    v = qrot_ref(hinv, s.ang);
    o[286 + b * 3 + 0] = v.x; o[286 + b * 3 + 1] = v.y; o[286 + b * 3 + 2] = v.z;
    float* t = o + HE_OBS_SELF;
    v = qrot_ref(hinv, r.pos - s.pos);
    t[b * 3 + 0] = v.x; t[b * 3 + 1] = v.y; t[b * 3 + 2] = v.z;
    f4 dq = qmul_ref(qmul_ref(hinv, qmul_ref(r.rot, qconj(s.rot))), hq);
    tan_norm(dq, tn);
#pragma unroll
    for (int c = 0; c < 6; ++c) t[72 + b * 6 + c] = tn[c];
    v = qrot_ref(hinv, r.vel - s.vel);
    t[216 + b * 3 + 0] = v.x; t[216 + b * 3 + 1] = v.y; t[216 + b * 3 + 2] = v.z;
    v = qrot_ref(hinv, r.ang - s.ang);
    t[288 + b * 3 + 0] = v.x; t[288 + b * 3 + 1] = v.y; t[288 + b * 3 + 2] = v.z;
    v = qrot_ref(hinv, r.pos - root_pos);
    t[360 + b * 3 + 0] = v.x; t[360 + b * 3 + 1] = v.y; t[360 + b * 3 + 2] = v.z;
    tan_norm(qmul_ref(hinv, r.rot), tn);
#pragma unroll
    for (int c = 0; c < 6; ++c) t[432 + b * 6 + c] = tn[c];
}

// humanoid_phc.py:694-731 + 747-780 + 901-931 for body b of env e: set the env to the
// reference state `r` (the blend at the reset time, offset = the env's pre-reset global offset,
// :858-860) and the dof state of the cold records `c` at the same frames. Every value written comes
// from registers: nothing is read back, so a reset costs no store -> load round trip.
HE_DEV void reset_body_write(const ImitArgs& a, int e, int b, const BodyRef& r, const ColdRows& x) {
    float* rb = a.rb_state + ((size_t)e * NB + b) * 13;
    const float row[13] = {r.pos.x, r.pos.y, r.pos.z, r.rot.x, r.rot.y, r.rot.z, r.rot.w,
                           r.vel.x, r.vel.y, r.vel.z, r.ang.x, r.ang.y, r.ang.z};
#pragma unroll
    for (int c = 0; c < 13; ++c) rb[c] = row[c];
    if (a.contact_forces) {
        float* cf = a.contact_forces + ((size_t)e * NB + b) * 3;
        cf[0] = cf[1] = cf[2] = 0.0f;
    }
    if (b == 0) {
        float* rs = a.root_states + (size_t)e * 13;
#pragma unroll
        for (int c = 0; c < 13; ++c) rs[c] = row[c];
    } else {
        f3 dp, dv;
        body_dof_blend(x, dp, dv);
        int d = 3 * (b - 1);
        float* ds = a.dof_state + ((size_t)e * ND + d) * 2;
        ds[0] = dp.x; ds[1] = dv.x; ds[2] = dp.y; ds[3] = dv.y; ds[4] = dp.z; ds[5] = dv.z;
        if (a.dof_targets) {
            float* tg = a.dof_targets + (size_t)e * ND + d;
            tg[0] = dp.x; tg[1] = dp.y; tg[2] = dp.z;
        }
    }
}

// The state init of a reset from its uniform draw u (include/humanoid_engine.h, he_sim_params'
// StateInit block; oracle/he_oracle.c resolve_init): true = a reference-state init at phase `ph`
// (humanoid_phc.py:694-731, 848-856), false = the initial pose (_reset_default, :688-692).
HE_DEV bool resolve_init(const he_imitation_params& p, float u, float& ph) {
#pragma clang fp contract(off)
    bool ref = p.state_init != HE_STATE_INIT_DEFAULT;
    ph = u;
    if (p.state_init == HE_STATE_INIT_HYBRID) {  // torch.bernoulli(hybrid_init_prob) (:733-745)
        ref = u < p.hybrid_init_prob;
        ph = ref ? u / p.hybrid_init_prob : 0.0f;
    }
    if (p.state_init == HE_STATE_INIT_START || p.test_mode) ph = 0.0f;
    return ref;
}

// _reset_default + _reset_env_tensors (humanoid_phc.py:688-692, 747-780) of body b of env e: the root
// row of HE_BUF_INIT_ROOT_STATE, zero dof positions / velocities / targets, and the rigid-body row of
// that pose (every local rotation the identity: the root rotation, origin root + R rest_pos[b]; the
// velocities of the initial root state, which the reference zeroes), zero contact force.
HE_DEV SimBody default_reset_body(const ImitArgs& a, int e, int b, bool act) {
#pragma clang fp contract(off)
    const float* irp = a.init_root + (size_t)e * 13;
    float ir[13];
#pragma unroll
    for (int c = 0; c < 13; ++c) ir[c] = irp[c];
    const f3 rp = f3{ir[0], ir[1], ir[2]};
    const f4 rq = f4{ir[3], ir[4], ir[5], ir[6]};
    const f3 v = f3{ir[7], ir[8], ir[9]}, w = f3{ir[10], ir[11], ir[12]};
    const f3 lo = f3{a.rest_pos[3 * b], a.rest_pos[3 * b + 1], a.rest_pos[3 * b + 2]};
    const f3 ro = qrot_ref(rq, lo);
    const f3 pos = rp + ro;
    const f3 vel = v + f3{w.y * ro.z - w.z * ro.y, w.z * ro.x - w.x * ro.z, w.x * ro.y - w.y * ro.x};
    if (act) {
        float* rb = a.rb_state + ((size_t)e * NB + b) * 13;
        rb[0] = pos.x; rb[1] = pos.y; rb[2] = pos.z;
        rb[3] = rq.x; rb[4] = rq.y; rb[5] = rq.z; rb[6] = rq.w;
        rb[7] = vel.x; rb[8] = vel.y; rb[9] = vel.z;
        rb[10] = w.x; rb[11] = w.y; rb[12] = w.z;
        if (a.contact_forces) {
            float* cf = a.contact_forces + ((size_t)e * NB + b) * 3;
            cf[0] = cf[1] = cf[2] = 0.0f;
        }
        if (b == 0) {
            float* rs = a.root_states + (size_t)e * 13;
#pragma unroll
            for (int c = 0; c < 13; ++c) rs[c] = ir[c];
        } else {
            const int d = 3 * (b - 1);
            float* ds = a.dof_state + ((size_t)e * ND + d) * 2;
            ds[0] = ds[1] = ds[2] = ds[3] = ds[4] = ds[5] = 0.0f;
            if (a.dof_targets) {
                float* tg = a.dof_targets + (size_t)e * ND + d;
                tg[0] = tg[1] = tg[2] = 0.0f;
            }
        }
    }
    return SimBody{pos, vel, w, rq};
}

// eval recording (he_imitation.hip; only the stand-alone kernel instantiates EVAL = true)
HE_DEV void eval_record(const he_eval_buffers& ev, int e, int lane, bool act, f3 p, f3 g);

// One env's reward / reset / termination / observation (and the fused device reset, mode 1) from
// its post-physics state: `s` = the lane's body row, `pw` = the lane's power-reward term
// (|tau . qdot| of its joint), mid / off / start / soff / prog = the env's motion bookkeeping as read
// before the step. `leader` is the lane that writes the env's scalars (group lane 0). Split in two
// so that the physics kernel can issue the reference loads (imitation_ref) long before the state
// they are compared with exists (imitation_finish).
// The part of the step that depends only on the env's bookkeeping: the motion metadata and both
// reference samples (t for the reward / reset, t + dt for the observation) of the lane's body.
struct ImitRef {
    int64_t mid;
    f3 off;
    float start, soff, t;
    int prog;
    MotionMeta mm;
    BodyRef r, r2;
};
// trip 2: the motion's metadata (the env's bookkeeping as read before the step)
struct ImitBook {
    int64_t mid;
    f3 off;
    float start, soff;
    int prog;
    MotionMeta mm;
};
HE_DEV ImitBook imitation_book(const ImitArgs& a, int64_t mid, f3 off, float start, float soff, int prog) {
    return ImitBook{mid, off, start, soff, prog, motion_meta(a.m, mid)};
}
// trip 3: both samples' frame records of the lane's body (loads), then their blends
struct ImitRaw {
    ImitBook k;
    int prog;
    float t;
    RefRows s1, s2;
};
HE_DEV ImitRaw imitation_frames_load(const ImitArgs& a, int lane, const ImitBook& k) {
    const int b = lane < NB ? lane : 0;
    const he_imitation_params& p = a.p;
    ImitRaw x;
    x.k = k;
    int prog = k.prog;
    if (a.mode != 2) prog += 1;  // post-physics half of HumanoidPHC.step (humanoid_phc.py:138-149)
    x.prog = prog;
    x.t = env_time(prog, p.control_dt, k.start, k.soff);
#if HE_IMIT_DIAG & 2  // frames at fixed indices: no dependent round trip
    x.s1 = body_ref_load(a.m, FrameSel{0, 1, x.t * 1e-9f}, b);
    x.s2 = body_ref_load(a.m, FrameSel{1, 2, x.t * 1e-9f}, b);
#else
    x.s1 = body_ref_load(a.m, frame_select(k.mm, x.t), b);
    x.s2 = body_ref_load(a.m, frame_select(k.mm, env_time(prog + 1, p.control_dt, k.start, k.soff)), b);
#endif
    return x;
}
HE_DEV ImitRef imitation_frames_blend(const ImitRaw& w) {
    ImitRef x;
    x.mid = w.k.mid; x.off = w.k.off; x.start = w.k.start; x.soff = w.k.soff;
    x.mm = w.k.mm;
    x.prog = w.prog;
    x.t = w.t;
    x.r = body_ref_blend(w.s1, w.k.off);
    x.r2 = body_ref_blend(w.s2, w.k.off);
    return x;
}
HE_DEV ImitRef imitation_frames(const ImitArgs& a, int lane, const ImitBook& k) {
    return imitation_frames_blend(imitation_frames_load(a, lane, k));
}
HE_DEV ImitRef imitation_ref(const ImitArgs& a, int lane, int64_t mid, f3 off, float start, float soff, int prog) {
    return imitation_frames(a, lane, imitation_book(a, mid, off, start, soff, prog));
}

template <bool EVAL>
HE_DEV void imitation_finish(const ImitArgs& a, int slot, int e, int lane, bool leader, const ImitRef& x, SimBody s,
                             float pw) {
    const bool act = lane < NB;
    const int b = act ? lane : 0;
    const he_imitation_params& p = a.p;
    f3 off = x.off;
    float start = x.start, soff = x.soff;
    int prog = x.prog;
    const MotionMeta mm = x.mm;
    const float t = x.t;
    const BodyRef r = x.r;
    BodyRef r2 = x.r2;
    bool do_reset = false, ref_init = true;
    float reset_time = 0.0f;

#if HE_IMIT_DIAG & 4  // no reward / termination math
    if (a.mode != 2) {
        if (leader) { a.rew[e] = r.pos.x + s.pos.x + pw + t; a.progress[e] = (int16_t)prog; }
    } else
#else
    if (a.mode != 2) {
#endif
#if !(HE_IMIT_DIAG & 4)
        // reward terms, common.py:298-317
        f3 d = r.pos - s.pos;
        float dp = act ? (d.x * d.x + d.y * d.y + d.z * d.z) / 3.0f : 0.0f;
        d = r.vel - s.vel;
        float dv = act ? (d.x * d.x + d.y * d.y + d.z * d.z) / 3.0f : 0.0f;
        d = r.ang - s.ang;
        float da = act ? (d.x * d.x + d.y * d.y + d.z * d.z) / 3.0f : 0.0f;
#if HE_IMIT_DIAG & 16
        float ang = qmul_ref(r.rot, qconj(s.rot)).w;
#else
        float ang = q_angle_axis(qmul_ref(r.rot, qconj(s.rot)), nullptr);
#endif
        float dr = act ? ang * ang : 0.0f;
        dp = group_sum(dp) / NB;
        dv = group_sum(dv) / NB;
        da = group_sum(da) / NB;
        dr = group_sum(dr) / NB;
        float rp = expf(-p.k_pos * dp), rr = expf(-p.k_rot * dr), rv = expf(-p.k_vel * dv), ra = expf(-p.k_ang_vel * da);
        float rew = p.w_pos * rp + p.w_rot * rr + p.w_vel * rv + p.w_ang_vel * ra;
        float pr = 0.0f;
        if (p.use_power_reward) {
            pw = group_sum(pw);
            pr = -p.power_coef * pw;
            if (prog <= 3) pr = 0.0f;
            rew += pr;
        }
        // termination, common.py:325-364 + humanoid_phc.py:1313-1335
        bool pass_time = t >= mm.len;
        bool fallen = false;
        if (p.enable_early_termination && !(HE_IMIT_DIAG & 32)) {
            bool inset = act && ((p.reset_body_mask >> b) & 1);
            float dist = norm3_im(s.pos - r.pos);  // no contraction in either TU (torch rounding)
            if (p.eval_mode) {
                float sum = group_sum(inset ? dist : 0.0f);
                float cnt = group_sum(inset ? 1.0f : 0.0f);
                int first = __ffs(p.reset_body_mask) - 1;
                fallen = cnt > 0.0f && (sum / cnt) > p.term_dist[first < 0 ? 0 : first];
            } else {
                fallen = group_max(inset && dist > p.term_dist[b] ? 1.0f : 0.0f) > 0.0f;
            }
            fallen = fallen && prog > 1;
        }
        bool reset = pass_time || fallen;
#if HE_IMIT_DIAG & 128  // no env resets at run time (the code stays)
        reset = reset && a.seed == 0x123456789abcdefull;
#endif
        if constexpr (EVAL) eval_record(a.ev, e, lane, act, s.pos, r.pos);  // before any fused reset
        if (leader) {
            a.rew[e] = rew;
            float* raw = a.reward_raw + (size_t)e * HE_REWARD_RAW;
            raw[0] = rp; raw[1] = rr; raw[2] = rv; raw[3] = ra; raw[4] = pr;
            a.reset[e] = reset;
            a.terminate[e] = fallen;
            a.progress[e] = (int16_t)prog;
        }
        if (a.mode == 1 && reset && !(HE_IMIT_DIAG & 64)) {
            do_reset = true;
            // the reset's draw: a hashed uniform, resolved by the state init (humanoid_phc.py:679-692,
            // 733-745, 848-856)
            float ph;
            ref_init = resolve_init(a.p, hash_uniform(a.seed, a.step, (uint32_t)e), ph);
            reset_time = ref_init ? sample_time_interval(ph, mm.len) : 0.0f;
        }
    } else {
#else
    {
#endif
        do_reset = !(HE_IMIT_DIAG & 64);
        float ph;
        ref_init = resolve_init(a.p, a.phases[slot], ph);
        reset_time = ref_init ? sample_time_interval(ph, mm.len) : 0.0f;
    }

    if (do_reset && !ref_init) {  // _reset_default: the motion bookkeeping stays (the group is uniform)
        // the next observation's frames are loaded alongside the initial pose (one round trip)
        const RefRows n2 = body_ref_load(a.m, frame_select(mm, env_time(1, p.control_dt, start, soff)), b);
        s = default_reset_body(a, e, b, act);  // the row this lane wrote
        r2 = body_ref_blend(n2, off);
        prog = 0;
        if (leader) {
            a.progress[e] = 0;
            if (a.mode == 2) { a.reset[e] = 0; a.terminate[e] = 0; }
        }
    } else if (do_reset) {  // the group's branch is uniform
        // the reset frames (hot and cold records) and the next observation's frames, loaded
        // together: one round trip (the metadata is the step's)
        const FrameSel fs = frame_select(mm, reset_time);
        const RefRows h0 = body_ref_load(a.m, fs, b);
        const ColdRows c0 = body_cold_load(a.m, fs, b);
        const RefRows n2 = body_ref_load(a.m, frame_select(mm, env_time(1, p.control_dt, reset_time, 0.0f)), b);
        const BodyRef r0 = body_ref_blend(h0, off);
        if (act) reset_body_write(a, e, b, r0, c0);
        s = SimBody{r0.pos, r0.vel, r0.ang, r0.rot};  // the row this lane wrote (lane b = 0's on idle lanes)
        r2 = body_ref_blend(n2, f3{0.f, 0.f, 0.f});
        off = f3{0.f, 0.f, 0.f};
        start = reset_time;
        soff = 0.0f;
        prog = 0;
        if (leader) {
            a.global_offset[3 * e] = 0.0f; a.global_offset[3 * e + 1] = 0.0f; a.global_offset[3 * e + 2] = 0.0f;
            a.start_times[e] = reset_time;
            a.start_offsets[e] = 0.0f;
            a.progress[e] = 0;
            if (a.mode == 2) { a.reset[e] = 0; a.terminate[e] = 0; }
        }
    }

    // ---------------- observations for the next step (humanoid_phc.py:937-961, 1063-1067)
    f3 root_pos = f3{bcast0(s.pos.x), bcast0(s.pos.y), bcast0(s.pos.z)};
    f4 root_rot = f4{bcast0(s.rot.x), bcast0(s.rot.y), bcast0(s.rot.z), bcast0(s.rot.w)};
    float h = calc_heading(root_rot);
    // quat_from_angle_axis(+-h, z): sinf is odd and cosf even (both evaluate |x| and restore the
    // sign), so the heading rotation is the inverse's z negated, bit for bit
    const f4 hinv = heading_quat(-h), hq = f4{0.f, 0.f, -hinv.z, hinv.w};
#if !(HE_IMIT_DIAG & 1)
    if (act) write_obs(a.obs + (size_t)e * HE_OBS_DIM, b, s, root_pos, hinv, hq, r2);
#else
    if (act && b == 0) a.obs[(size_t)e * HE_OBS_DIM] = hinv.z + root_pos.z + r2.pos.x + s.vel.x;
#endif
}

// the power-reward term of joint `lane` (humanoid_phc.py:1297-1305): |tau . qdot| over its 3 dofs,
// f = the joint's 3 dof forces, v = its 3 dof velocities (stride vs between them)
HE_DEV float power_term(const float* f, const float* v, int vs) {
    return fabsf(f[0] * v[0]) + fabsf(f[1] * v[vs]) + fabsf(f[2] * v[2 * vs]);
}
