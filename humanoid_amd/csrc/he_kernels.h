// he_kernels.h -- kernel argument blocks and launchers shared by the engine TU and kernel TUs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/humanoid_engine.h"
#include "he_topo.h"

int he_fail_text(const char* text);  // sets he_last_error(), returns 1

#define HE_MOTION_HOT 13   // per body: pos3 rot4 vel3 angvel3 (same layout as a rigid-body row)
#define HE_MOTION_COLD 8   // per body: local rot4, dof vel3, pad

// device motion library: interleaved per-frame records
struct MotionDev {
    const float* hot;             // [F][24][13]
    const float* cold;            // [F][24][8]
    const int64_t* length_starts; // [M]
    const int64_t* num_frames;    // [M]
    const float* lengths;         // [M]
    const float* dt;              // [M]
    int num_motions;              // M (ids are clamped into range: a bad id must never fault)
};

struct ImitArgs {
    he_imitation_params p;
    MotionDev m;
    float* root_states;      // [N,13]
    float* dof_state;        // [N,69,2]
    float* rb_state;         // [N,24,13]
    float* contact_forces;   // [N,24,3]
    const float* dof_force;  // [N,69]
    float* dof_targets;      // [N,69]
    const int64_t* motion_ids;
    float* start_times;
    float* start_offsets;
    float* global_offset;
    int16_t* progress;
    float* obs;
    float* rew;
    float* reward_raw;
    uint8_t* reset;
    uint8_t* terminate;
    const int32_t* env_ids;  // null = all envs [0, count)
    int count;
    int mode;                // 0 step, 1 step + fused device reset, 2 reset listed envs
    const float* phases;     // mode 2: [count]
    uint64_t seed, step;
    he_eval_buffers ev;      // eval recording (modes 0/1) when has_eval
    int has_eval;
    const float* init_root;  // [N,13] HE_BUF_INIT_ROOT_STATE (the Default / Hybrid state init)
    const float* rest_pos;   // [24,3] body origins of the zero pose in the root frame (model)
    int32_t* meta_cache;     // [N,8] per-env motion metadata (motion id, length, dt, frames, start) of the
                             // last step; null = read the motion tables every step
};

// AMP observation update, launched after an imitation launch
struct AmpArgs {
    MotionDev m;
    const float* rb_state;    // [N,24,13]
    const float* dof_state;   // [N,69,2]
    const int64_t* motion_ids;
    const float* start_times;
    const uint8_t* reset;     // mode 1: envs reset by the preceding launch
    const int32_t* env_ids;   // mode 2: the reset envs; null = all envs [0, count)
    int count;
    int mode;                 // 0 step update, 1 step update or init by reset flag, 2 init listed envs
    float control_dt;
    he_amp_buffers amp;
    // the reset draw of each env (modes 1 / 2), to tell a Default init (history = the current row,
    // _init_amp_obs_default) from a reference one (history from the motion)
    he_imitation_params ip;
    const float* phases;      // mode 2: [count]
    uint64_t seed, step;
    // function-level form (he_amp_observations): explicit inputs, K rows into `out`
    const float *root_pos, *root_rot, *root_vel, *root_ang_vel, *dof_pos, *dof_vel, *key_pos;
    float* out;
};

struct MotionStateArgs {
    MotionDev m;
    int k;
    const int64_t* ids;
    const float* times;
    const float* offset;
    float *rg_pos, *rb_rot, *body_vel, *body_ang_vel, *dof_pos, *dof_vel;
};

struct PhysArgs {
    he_sim_params p;
    const he_model* model;   // device copy
    const PhysTopo* topo;    // device copy
    float* root_states;
    float* dof_state;
    float* dof_targets;
    const float* actions;    // non-null: targets = offset + scale*clip(a) (frozen dofs 0) first
    const float* pd_offset;  // [69]
    const float* pd_scale;   // [69]
    const int32_t* frozen;   // [69]
    int clip_actions;
    float* rb_state;
    float* contact_forces;
    float* dof_force;
    int32_t* num_contacts;
    int32_t* dropped;            // [N] contacts generated past the capacity (last substep) or null
    float* cache;                // [N,HE_CACHE_WORDS] warm-start cache or null
    const float* mass_scale;     // [N,24] or null
    const float* friction;       // [N] or null
    const int32_t* terrain_kind; // [N] or null
    int num_envs;
    int substeps;
    unsigned long long* stamps;  // diagnostics: [N][16] phase cycles or null
    const int32_t* order;        // [N] env of each workgroup (launch_physics_order), or null: env = workgroup id
    uint32_t* cost;              // [N] each env's cycles in this launch (for launch_physics_order), or null
    int fused;                   // 1: the imitation step (mode 1) runs in the epilogue (he_env_step)
    int full_dofs;               // 1: no leg class (every env's Zh products over 75 dofs; HE_TGS_LEGS=0, tests)
    ImitArgs im;                 // its arguments when fused
};

hipError_t launch_imitation(const ImitArgs& a, hipStream_t stream);
hipError_t launch_amp(const AmpArgs& a, hipStream_t stream);
hipError_t launch_amp_function(const AmpArgs& a, hipStream_t stream);
hipError_t launch_motion_state(const MotionStateArgs& a, hipStream_t stream);
hipError_t launch_physics(const PhysArgs& a, hipStream_t stream);
// The physics launch's dispatch order, heavy envs first. A launch's 4096 one-wave workgroups fill the
// chip's 2048 wave slots twice, and the hardware hands the second round out in workgroup order as
// slots free: an expensive env dispatched late sets the launch's end. One 1024-thread workgroup reads
// the envs' cycle counts of the last launch (PhysArgs.cost) and writes order[] as a partition into
// 32 classes of cost / mean (steps of 1/32 from 0.5 to 1.5), the costliest class first: a
// longest-first order, so the slots that finish their first env early take the costly second-round
// envs and the costliest envs' slots take the cheapest last. Results do not depend on the order (envs
// never interact). The engine runs it every few physics launches (he_engine.cpp).
hipError_t launch_physics_order(const uint32_t* cost, int32_t* order, int num_envs, hipStream_t stream);
// First-dispatch warm-up (he_create_envs): every product kernel of the TU launched once with no work
// (count 0, one block that exits at its guard), so the one-time first-dispatch cost of each kernel
// (~0.4-0.8 ms on the MI355X, 16-30 ms under rocprofv3's kernel tracing) is paid at engine
// creation, not by the setup's first reset or a timed step. mode 1: one trivial kernel per TU
// (diagnostic: whether the cost is per code object or per kernel).
hipError_t warm_imitation_kernels(hipStream_t stream, int mode);
hipError_t warm_physics_kernels(hipStream_t stream, int mode);
hipError_t warm_ingest_kernels(hipStream_t stream, int mode);
bool physics_phase_stamps();  // built with HE_PHASE_STAMPS (diagnostic twin library)
hipError_t launch_ingest(const float* pose, const float* trans, const int32_t* parents, const float* local_pos,
                         const int64_t* starts, const int64_t* nframes, const float* dt, int num_clips, int64_t F,
                         float* hot, float* cold, float* gav_raw, hipStream_t stream);
