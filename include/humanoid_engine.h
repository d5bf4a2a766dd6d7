/*
 * humanoid_engine.h -- C ABI of libhumanoid_engine.so, the MI355X (gfx950) batched SMPL-humanoid
 * rollout engine that replaces Isaac Gym/PhysX + gymtorch under puffer-phc.
 *
 * Conventions
 *   - every entry point returns 0 on success, non-zero on failure; he_last_error() gives the text
 *     (the gymtorch C++ it replaces printf'ed and returned an empty tensor,
 *      packages/gymtorch/gymtorch/gymtorch.cpp:40-51,114-117; the Python shim raises instead);
 *   - all float/int pointers passed to compute entry points are DEVICE pointers on the handle's
 *     device; `stream` is a hipStream_t (NULL = default stream); nothing here synchronises the host;
 *   - quaternions are xyzw (puffer_phc/torch_utils.py:61), Z-up, gravity -9.81 z
 *     (puffer_phc/envs/isaacgym_env.py:29-33).
 *
 * Each entry point cites the reference interface it replaces (paths under packages/puffer-phc/
 * unless noted). Isaac Gym's own binary is not vendored; the cited lines are its call sites.
 */
#ifndef HUMANOID_ENGINE_H
#define HUMANOID_ENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HE_NUM_BODIES 24
#define HE_NUM_DOF 69
#define HE_NUM_GEN 75          /* 6 root + 69 joint generalized velocities */
#define HE_MAX_PAIRS 256
#define HE_STAMP_SLOTS 32 /* diagnostic per-phase cycle slots per env (he_set_debug_stamps) */
#define HE_MAX_CONTACTS 40       /* contact slots (points, joint limits) per env */
#define HE_MAX_ROWS 63           /* solver rows per env, one per lane of a 64-lane wave: a joint limit
                                    1, a point 1 normal row, its friction on its patch (patch friction:
                                    2 tangential rows per body-terrain patch and, from 2 points on, 1
                                    torsional row; a self pair 2 tangential rows of its own) */
#define HE_OBS_SELF 358
#define HE_OBS_TASK 576
#define HE_OBS_DIM 934         /* humanoid_phc.py:458-467 */
#define HE_REWARD_RAW 5        /* 4 imitation terms + power, humanoid_phc.py:562-569 */

/* geometry kinds (one geom per body, assets/smpl_humanoid.xml:27-168) */
#define HE_GEOM_SPHERE 0
#define HE_GEOM_CAPSULE 1
#define HE_GEOM_BOX 2

/* Model blob: what gym.load_asset + get_asset_dof_properties + create_actor give the reference
 * (humanoid_phc.py:211-230, 276-324, 370-381). Built on the host from the MJCF. */
typedef struct he_model {
    int32_t num_bodies, num_dof, num_pairs, reserved;
    int32_t parents[HE_NUM_BODIES];
    int32_t geom_type[HE_NUM_BODIES];
    float local_pos[HE_NUM_BODIES][3];   /* joint offset in parent frame */
    float mass[HE_NUM_BODIES];
    float com[HE_NUM_BODIES][3];         /* body frame */
    float inertia[HE_NUM_BODIES][6];     /* about COM, body frame: xx yy zz xy xz yz */
    float geom_params[HE_NUM_BODIES][10];
    float geom_radius[HE_NUM_BODIES];
    float stiffness[HE_NUM_DOF], damping[HE_NUM_DOF], armature[HE_NUM_DOF], effort[HE_NUM_DOF];
    int32_t pairs[HE_MAX_PAIRS][2];      /* self-collision candidate pairs */
    /* dof ranges (rad) from the MJCF joint ranges (get_asset_dof_properties lower/upper,
     * humanoid_phc.py:305-324), enforced on the exp-map coordinates when joint_limits is set */
    float dof_lower[HE_NUM_DOF], dof_upper[HE_NUM_DOF];
} he_model;

/* Simulation parameters: isaacgym_env.py:6-35 + asset options humanoid_phc.py:211-214. */
typedef struct he_sim_params {
    float dt;                        /* 1/60 */
    float gravity[3];                /* 0 0 -9.81 */
    float contact_offset;            /* 0.02 */
    float friction;                  /* 1.0 (plane static=dynamic=1, humanoid_phc.py:259-260) */
    float baumgarte;                 /* penetration recovery fraction per substep */
    float max_depenetration_velocity;/* 10 */
    float angular_damping;           /* 0.01 */
    float max_angular_velocity;      /* 100 */
    int32_t solver_iterations;       /* PGS sweeps per substep */
    int32_t self_collision;          /* 1 = has_self_collision (config.py:57) */
    int32_t max_contacts;            /* contact slots, <= HE_MAX_CONTACTS (rows are capped at
                                        HE_MAX_ROWS whatever this is) */
    float kp_scale, kd_scale;        /* config.py:106-107 */
    int32_t terrain;                 /* 0 plane everywhere, 1 per-env terrain kind (config 5) */
    float terrain_slope;             /* radians, terrain kind 1 */
    float step_height, step_length;  /* terrain kind 2 (box steps along +x) */
    int32_t joint_limits;            /* 1: unilateral limit rows on the dof ranges (PhysX limits) */
    float limit_margin;              /* rad: a limit row is emitted within margin + dt*closing rate */
    int32_t warm_start;              /* 1: the solver starts from the previous solve's impulses */
    float solver_tolerance;          /* m/s: stop the sweeps once no row's velocity moves by more
                                        (|d lambda_r| A_rr) in a sweep; 0 = always solver_iterations */
    int32_t bias_midpoint;           /* 1 (default): the velocity-dependent bias (Coriolis,
                                        gyroscopic) evaluated at the midpoint velocity (u0 + uf) / 2
                                        of the explicit step, one more solve through the same factor
                                        (explicit at dt 1/120 pumps energy under
                                        per-step random targets); 0: explicit, at u0 */
    int32_t substeps;                /* gymapi.SimParams.substeps (Isaac Gym default 2; the reference
                                        leaves it, isaacgym_env.py:6-35): each simulate() advances dt
                                        in `substeps` physics steps of dt / substeps */
    float max_joint_velocity;        /* rad/s, per joint relative rate (PhysX articulation joint
                                        maxJointVelocity, default 100); max_angular_velocity above
                                        clamps each link's WORLD angular velocity (PxRigidBody) */
    int32_t solver_type;             /* sim_params.physx.solver_type (isaacgym_env.py:16): 0 PGS --
                                        `solver_iterations` velocity-level Gauss-Seidel sweeps per
                                        physics step; 1 TGS -- `solver_iterations` position iterations
                                        (num_position_iterations, :17) inside each physics step of dt:
                                        the step's factor and contact set are kept, and iteration k is
                                        one sweep at the sub-step h = dt / solver_iterations against the
                                        separations advanced by h J u_j of the earlier iterations; the
                                        positions advance by the sub-steps' mean velocity, the step ends
                                        at the last iteration's (DESIGN.md §5 "TGS") */
} he_sim_params;

/* Per-env solver warm-start cache (f32 words; HE_BUF_CONTACT_CACHE), written at the end of every
 * step and read at the start of the next when the env's root pose still equals the signature
 * (any external state write -- a reset -- invalidates it). It holds the last solve's rows:
 *   [0,7)   signature: root position, root quaternion as written by the step
 *   7       number of cached rows (int32 bits)
 *   [8,40)  row keys, 16 bits each, row 2j in the low half of word 8 + j, row 2j+1 in the high half:
 *           body0 | (body1 + 2) << 5 | sub << 10 | kind << 14 with body1 = -1 terrain (sub = the
 *           point: capsule end / box corner; HE_KEY_PATCH for the friction rows of the body's
 *           terrain patch), -2 joint limit (sub = 1 + 2 axis + side, 7 the rotation angle), else
 *           the self-collision partner (sub = 0); kind 0 normal, 1 and 2 tangential, 3 torsional
 *   [40,40+HE_MAX_ROWS)  the rows' impulses */
#define HE_CACHE_WORDS 104
#define HE_CACHE_KEYS 8
#define HE_CACHE_LAMBDA 40
#define HE_KEY_PATCH 15

/* Imitation (reward / reset / obs) parameters: config.py:37-50, 97-112; humanoid_phc.py:1230-1335. */
typedef struct he_imitation_params {
    float k_pos, k_rot, k_vel, k_ang_vel;
    float w_pos, w_rot, w_vel, w_ang_vel;
    float power_coef;                /* rew_power_coef 0.0005 */
    int32_t use_power_reward;        /* 1 */
    float control_dt;                /* isaac_base.dt = 2 * 1/60 */
    int32_t enable_early_termination;/* 1 */
    int32_t eval_mode;               /* flag_im_eval: mean-distance termination */
    int32_t reset_body_mask;         /* bit b set = body b in _reset_bodies_id */
    float term_dist[HE_NUM_BODIES];  /* _termination_distances */
    int32_t state_init;              /* StateInit (envs/state_init.py; config.py:114 default Random):
                                        0 Default: the initial pose (humanoid_phc.py:688-692),
                                        1 Start: the reference state at motion time 0,
                                        2 Random: at sample_time_interval of the phase (:848-852),
                                        3 Hybrid: Bernoulli(hybrid_init_prob) Random, else Default
                                        (:733-745) */
    float hybrid_init_prob;          /* config.py:139 */
    int32_t test_mode;               /* flag_test: reference-state inits at motion time 0 (:855-856) */
    int32_t reserved;
} he_imitation_params;

/* StateInit values (envs/state_init.py) */
#define HE_STATE_INIT_DEFAULT 0
#define HE_STATE_INIT_START 1
#define HE_STATE_INIT_RANDOM 2
#define HE_STATE_INIT_HYBRID 3
/* How a reset turns its uniform draw u in [0,1) (he_reset_envs' `phases`, or the device reset's
 * hash) into the state init, identically in the kernels and the oracle: Default -> the initial
 * pose; Start -> reference at t = 0; Random -> reference at sample_time_interval(u); Hybrid -> the
 * reference at sample_time_interval(u / p) when u < p = hybrid_init_prob (u / p is uniform given
 * the draw), else the initial pose; test_mode puts every reference init at t = 0. */

/* Buffer kinds (humanoid_phc.py:497-554, the tensors gymtorch.wrap_tensor exposed). */
typedef enum he_buf_kind {
    HE_BUF_ROOT_STATE = 0,     /* f32 [N,13]  pos3 quat4 linvel3 angvel3  (acquire_actor_root_state_tensor) */
    HE_BUF_DOF_STATE = 1,      /* f32 [N*69,2] (pos, vel)                 (acquire_dof_state_tensor) */
    HE_BUF_RB_STATE = 2,       /* f32 [N*24,13]                           (acquire_rigid_body_state_tensor) */
    HE_BUF_CONTACT_FORCE = 3,  /* f32 [N*24,3]                            (acquire_net_contact_force_tensor) */
    HE_BUF_DOF_FORCE = 4,      /* f32 [N*69]                              (acquire_dof_force_tensor) */
    HE_BUF_DOF_TARGET = 5,     /* f32 [N,69]  position targets            (set_dof_position_target_tensor) */
    HE_BUF_NUM_CONTACTS = 6,   /* i32 [N]     contact slots used last substep (limits included) */
    HE_BUF_DROPPED_CONTACTS = 7, /* i32 [N]   contacts generated past the capacity, last substep */
    HE_BUF_CONTACT_CACHE = 8,  /* f32 [N,HE_CACHE_WORDS] solver warm-start cache (see above) */
    HE_BUF_INIT_ROOT_STATE = 9, /* f32 [N,13] _initial_humanoid_root_states (humanoid_phc.py:522-523):
                                  the creation poses with zero velocities, set by he_create_envs
                                  (z = 0.89, identity rotation, start_xy); writable: the gym
                                  facade's prepare_sim writes the actors' own creation poses
                                  here when they differ; the Default / Hybrid state init resets
                                  to it */
    HE_BUF_PHYS_ORDER = 10,    /* i32 [N] the physics launch's dispatch order: the env of each workgroup,
                                  expensive envs first (engine extension, read-only diagnostics;
                                  rebuilt every HE_PHYS_ORDER launches, default 8) */
    HE_BUF_PHYS_COST = 11,     /* i32 [N] each env's wave cycles in the last physics launch (the order's
                                  input; read-only diagnostics) */
    HE_BUF_COUNT = 12
} he_buf_kind;

#define HE_DTYPE_F32 1   /* GymTensor.h:23 eGymDataTypeFp32 */
#define HE_DTYPE_I32 2   /* GymTensor.h:24 eGymDataTypeUint32 (torch int32) */

typedef struct he_engine he_engine;

const char* he_last_error(void);
int he_version(void);
int he_device_count(int* count);

/* gymapi.acquire_gym + create_sim (isaacgym_env.py:48-50): bind a HIP device, copy params. */
int he_create(const he_sim_params* params, int device, he_engine** out);
/* gym.load_asset (humanoid_phc.py:216); the host parses the MJCF into the blob. Fails (with the
 * reason in he_last_error) on a topology other than 24 bodies / 69 dofs in DFS order, more than
 * HE_MAX_PAIRS self pairs or more than 5 box geoms (the kernel's corner lanes; SMPL has 4). */
int he_set_model(he_engine* h, const he_model* model);
/* create_env/create_actor x N + prepare_sim (humanoid_phc.py:264-326, :74): allocates the state
 * tensors, places actors at (start_xy, 0.89) with identity rotation (humanoid_phc.py:340-347). */
int he_create_envs(he_engine* h, int num_envs, const float* host_start_xy);
/* gym.destroy_sim (isaacgym_env.py:99) */
int he_destroy(he_engine* h);

/* acquire_*_tensor (humanoid_phc.py:499-504): device pointer + shape of an engine-owned buffer.
 * The memory stays owned by the engine (non-owning wrap, gymtorch.cpp:90). */
int he_get_buffer(he_engine* h, int kind, void** dptr, int64_t* shape, int* ndim, int* dtype);

/* set_dof_position_target_tensor (humanoid_phc.py:127-128): device-to-device copy of [N,69]. */
int he_set_dof_targets(he_engine* h, const float* src, void* stream);
/* set_{actor_root_state,dof_state,dof_position_target}_tensor_indexed (humanoid_phc.py:750-767):
 * rows `ids[0..k)` (int32 actor ids = env ids, one actor per env) are copied from the full-size
 * source tensor into the engine state. */
int he_set_root_state_indexed(he_engine* h, const float* src, const int32_t* ids, int k, void* stream);
int he_set_dof_state_indexed(he_engine* h, const float* src, const int32_t* ids, int k, void* stream);
int he_set_dof_targets_indexed(he_engine* h, const float* src, const int32_t* ids, int k, void* stream);

/* Per-env domain randomisation (config 5; the reference removed it, humanoid_phc.py:349):
 * body mass scale [N,24] and friction [N], terrain kind [N] (0 plane, 1 slope, 2 steps).
 * NULL disables the corresponding array. Device pointers, owned by the caller. */
int he_set_env_properties(he_engine* h, const float* mass_scale, const float* friction,
                          const int32_t* terrain_kind);

/* gym.simulate x num_simulate + fetch_results (humanoid_phc.py:131-134; num_simulate =
 * control_freq_inv = 2 per policy step): articulated rigid-body step with implicit PD drives,
 * ground + self contacts and a PGS contact solve, num_simulate x he_sim_params.substeps physics
 * steps of dt / substeps; updates every state buffer (root, dof, rigid-body, contact force, dof
 * force). One kernel launch. */
int he_simulate(he_engine* h, int num_simulate, void* stream);
/* action -> PD target (humanoid_phc.py:1218-1228, freeze hand/toe :116-125) fused into the step:
 * target = offset + scale*clip(a,-1,1) (frozen dofs 0), then he_simulate. */
int he_set_pd_params(he_engine* h, const float* host_offset, const float* host_scale,
                     const int32_t* host_frozen_mask, int clip_actions);
int he_step_actions(he_engine* h, const float* actions, int num_simulate, void* stream);
/* refresh_*_tensor (humanoid_phc.py:782-789): buffers are the live engine state, nothing to copy;
 * kept for API parity (no FK recompute: rigid-body rows written by the caller after a reset stay,
 * as the reference relies on, humanoid_phc.py:922-931). */
int he_refresh(he_engine* h, void* stream);

/* ---------------- motion library + fused imitation kernel (A5-A9) ---------------------- */
/* MotionLibBase.load_motions table upload (motion_lib.py:396-420). Host pointers; the engine
 * re-lays the frames out as interleaved per-frame records in device memory.
 * gts/gvs/gavs [F,24,3], grs/lrs [F,24,4], dvs [F,23,3]; per-motion arrays [M]. */
int he_load_motions(he_engine* h, int64_t num_frames_total, int num_motions,
                    const float* gts, const float* grs, const float* lrs, const float* gvs,
                    const float* gavs, const float* dvs, const int64_t* length_starts,
                    const int64_t* num_frames, const float* lengths, const float* dt);

/* Device-side motion ingestion: replaces the host MotionLibSMPL.load_motions
 * path (motion_lib.py:257-429, 743-824 with poselib_skeleton.py:518-539, 574-592, 1166-1251 and
 * compute_motion_dof_vels_jit motion_lib.py:119-140). Clips are concatenated along frames:
 * pose_quat_global [F,24,4] xyzw and root_trans [F,3] (the .pkl schema's pose_quat_global /
 * root_trans_offset), DEVICE pointers; host_num_frames / host_fps [num_clips] HOST arrays. Builds
 * the motion tables on the device (local rotations, FK translations, Gaussian-filtered linear and
 * angular velocities, dof velocities). Motion i of the library refers to clip
 * host_motion_clip[i] (HOST, [num_motions]; NULL = identity with num_motions = num_clips), as the
 * reference's per-env motion entries share clips. Synchronises `stream`. */
int he_ingest_clips(he_engine* h, int num_clips, const int64_t* host_num_frames, const float* host_fps,
                    const float* pose_quat_global, const float* root_trans, int num_motions,
                    const int32_t* host_motion_clip, void* stream);

/* Per-env motion bookkeeping buffers (device, caller-owned, all [N] unless noted):
 * motion_ids i64, start_times f32, start_offsets f32, global_offset f32 [N,3], progress i16. */
typedef struct he_env_motion {
    const int64_t* motion_ids;
    float* start_times;
    float* start_offsets;
    float* global_offset;
    int16_t* progress;
} he_env_motion;

/* Post-physics half of HumanoidPHC.step (humanoid_phc.py:138-149): progress += 1, then
 * _compute_reward (:1230-1305), _compute_reset (:1313-1335) and _compute_observations
 * (:937-961) for all envs, in one launch. Outputs: obs [N,934], rew [N], reward_raw [N,5],
 * reset u8 [N], terminate u8 [N]. */
int he_imitation_step(he_engine* h, const he_imitation_params* p, const he_env_motion* em,
                      float* obs, float* rew, float* reward_raw, uint8_t* reset, uint8_t* terminate,
                      void* stream);

/* MotionLibBase.get_motion_state (motion_lib.py:549-626) for K queries (device arrays):
 * ids i64 [K], times f32 [K], offset f32 [K,3] or NULL. Outputs (device, nullable):
 * rg_pos [K,24,3], rb_rot [K,24,4], body_vel [K,24,3], body_ang_vel [K,24,3],
 * dof_pos [K,69], dof_vel [K,69]. */
int he_motion_state(he_engine* h, int k, const int64_t* ids, const float* times, const float* offset,
                    float* rg_pos, float* rb_rot, float* body_vel, float* body_ang_vel,
                    float* dof_pos, float* dof_vel, void* stream);

/* _reset_actors + _reset_env_tensors + _compute_observations(env_ids) (humanoid_phc.py:665-692,
 * 694-745, 747-780, 937-961) for env ids [k] (int32), with `phases` f32 [k] uniform [0,1) resolved
 * by p->state_init (above). A reference-state init: motion time t = floor(phase*len/(1/30))*(1/30)
 * (motion_lib.py:526-535); writes root/dof/rigid-body state, dof targets := dof_pos, zero contact
 * forces, progress = 0, start_times = t, start_offsets = 0, global_offset = 0. A Default init
 * (_reset_default): root := HE_BUF_INIT_ROOT_STATE row, dof pos / vel / targets := 0, the
 * rigid-body rows of that pose (zero velocities), zero contact forces, progress = 0, the motion
 * bookkeeping left as it was (the reference does not touch it). Then the k obs rows. */
int he_reset_envs(he_engine* h, const he_imitation_params* p, const he_env_motion* em,
                  const int32_t* env_ids, int k, const float* phases, float* obs, uint8_t* reset,
                  uint8_t* terminate, void* stream);

/* Fully device-side env step used by the rollout path (no host sync): actions -> PD targets ->
 * physics -> reward/reset/obs -> device reset of flagged envs (phases from a counter-based hash
 * of (seed, step, env)) -> obs for reset envs. */
int he_env_step(he_engine* h, const he_imitation_params* p, const he_env_motion* em,
                const float* actions, int num_simulate, uint64_t seed, uint64_t step_index,
                float* obs, float* rew, float* reward_raw, uint8_t* reset, uint8_t* terminate,
                void* stream);

/* he_env_step as ONE launch (the imitation step in the physics kernel's epilogue) or as two
 * (he_step_actions + he_imitation_reset_step): enable 1 / 0, or -1 = auto (the default: one launch
 * up to 2048 envs, where launch and tail latency dominate). Eval recording always takes two. Both
 * forms give the same results bit for bit (tests/test_gpu_parity.py). */
int he_set_fused_step(he_engine* h, int enable);

/* Second half of he_env_step on its own (after he_step_actions): reward/reset/obs with the device
 * reset of flagged envs. he_env_step == he_step_actions + he_imitation_reset_step. */
int he_imitation_reset_step(he_engine* h, const he_imitation_params* p, const he_env_motion* em, uint64_t seed,
                            uint64_t step_index, float* obs, float* rew, float* reward_raw, uint8_t* reset,
                            uint8_t* terminate, void* stream);

/* Eval-mode metric recording. While attached, every imitation launch that steps
 * (he_imitation_step, he_imitation_reset_step, he_env_step) also records, per env and before any
 * fused reset, what the reference copies to the host each eval step (humanoid_phc.py:158-169:
 * extras "mpjpe", "body_pos", "body_pos_gt") and accumulates the per-frame metrics that
 * EvalStats.get_final_stats computes over the stacked copies with smpl_sim's compute_metrics_lite
 * (scripts/phc_train.py:126-128, 166-189; smpl_sim 0.0.1 @ fe22a5d9, un-vendored): mpjpe_g,
 * mpjpe_l, mpjpe_pa, vel_dist, accel_dist in mm. Frame `frame` (EvalStats.curr_steps) of env e
 * counts while frame < num_steps[e] - 1 (the `[: (i - 1)]` slices, phc_train.py:146-151); frame 0
 * restarts the env's sums. sums[e] = {mpjpe_g, mpjpe_l, mpjpe_pa, vel_dist, accel_dist} summed over
 * counted frames, then {n_frames, n_vel, n_accel}. */
#define HE_EVAL_SUMS 8
typedef struct he_eval_buffers {
    const int32_t* num_steps;  /* [N] get_motion_num_steps() of each env's motion */
    float* mpjpe;              /* [N] extras["mpjpe"] (m), NULL to skip */
    float* body_pos;           /* [N,24,3] extras["body_pos"], NULL to skip */
    float* body_pos_gt;        /* [N,24,3] extras["body_pos_gt"], NULL to skip */
    float* history;            /* [N,2,2,24,3] scratch: the last two frames (pred, gt) */
    double* sums;              /* [N,HE_EVAL_SUMS] */
    int32_t frame;
    int32_t reserved;
} he_eval_buffers;

/* Attach (copied by value; call again each step with the new frame) or detach (NULL). */
int he_set_eval(he_engine* h, const he_eval_buffers* buffers);

/* ---------------- AMP observations (off by default, config.py:98) ------------ */
/* One AMP row (humanoid_phc.py:471-476 with has_dof_subset): root height 1, root rotation
 * tan-norm 6, local root velocity 3 and angular velocity 3, tan-norm of the 19 kept joints'
 * exp maps 114, their dof velocities 57, key-body positions 12 (body_sets.py:42-45). */
#define HE_AMP_OBS_STEP 196
#define HE_AMP_MAX_STEPS 64

/* _amp_obs_buf / _amp_obs_demo_buf (humanoid_phc.py:600-611), DEVICE pointers owned by the
 * caller, f32 [N, num_steps, 196] contiguous and 16-byte aligned: row 0 is the current AMP
 * observation, rows 1.. the history (the `amp_obs` [N, 1960] view the trainer stores,
 * clean_pufferl/core.py:174). */
typedef struct he_amp_buffers {
    float* amp_obs;       /* required */
    float* amp_obs_demo;  /* NULL to skip the demo copy */
    int32_t num_steps;    /* cfg.num_amp_obs_steps (config.py:141), 1..HE_AMP_MAX_STEPS */
    int32_t reserved;
} he_amp_buffers;

/* Attach (copied by value) or detach (NULL). While attached, every imitation launch is followed
 * by the AMP launch on the same stream:
 *  - he_imitation_step: _update_hist_amp_obs + _compute_amp_observations for every env
 *    (humanoid_phc.py:154-157, 1125-1176, 1341-1347): rows shift by one, row 0 from the state;
 *  - he_reset_envs: _init_amp_obs for the listed envs (humanoid_phc.py:665-676, 791-838):
 *    row 0 from the reset state, row k from the env's motion at start_time - k*dt (no offset),
 *    then amp_obs_demo[env] = amp_obs[env];
 *  - he_imitation_reset_step / he_env_step: the step update for envs not reset in the launch,
 *    the init for those that were. */
int he_set_amp(he_engine* h, const he_amp_buffers* buffers);

/* build_amp_observations_smpl (envs/common.py:191-267) with the flags humanoid_phc.py:1195-1210
 * passes, on K device rows: root_pos/vel/ang_vel [K,3], root_rot [K,4], dof_pos/dof_vel [K,69],
 * key_body_pos [K,4,3] (R_Ankle, L_Ankle, R_Wrist, L_Wrist) -> out [K,196]. No engine needed. */
int he_amp_observations(int k, const float* root_pos, const float* root_rot, const float* root_vel,
                        const float* root_ang_vel, const float* dof_pos, const float* dof_vel,
                        const float* key_body_pos, float* out, void* stream);

/* Diagnostics: when non-NULL, the physics kernel accumulates per-phase shader cycles into
 * device_buffer [N][HE_STAMP_SLOTS] (u64; phases listed in DESIGN.md §4). NULL disables (default).
 * Only the diagnostic twin library (libhumanoid_engine_phases.so) carries the stamps; the product
 * library returns nonzero for a non-NULL buffer. */
int he_set_debug_stamps(he_engine* h, uint64_t* device_buffer);

/* hash-based uniform used by he_env_step (exposed for parity tests): out[k] for env ids[k]. */
float he_hash_uniform(uint64_t seed, uint64_t step_index, uint32_t env);

#ifdef __cplusplus
}
#endif
#endif /* HUMANOID_ENGINE_H */
