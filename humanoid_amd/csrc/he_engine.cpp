// he_engine.cpp -- C-ABI implementation of libhumanoid_engine.so (include/humanoid_engine.h).
// Owns the device state (hipMalloc), the device model/topology blobs and the device motion
// library, and launches the gfx950 kernels on the caller's stream. No host synchronisation on
// any compute entry point; allocation happens only in he_create_envs / he_load_motions.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/humanoid_engine.h"
#include "he_kernels.h"
#include "he_topo.h"

size_t physics_lds_bytes();

namespace {
thread_local std::string g_err;

int fail(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return 1;
}

}  // namespace

// error text for the other C-ABI translation units (he_rollout.hip)
int he_fail_text(const char* text) {
    g_err = text;
    return 1;
}

namespace {
#define HE_CHECK(expr)                                                                         \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess) return fail("%s: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
    } while (0)

template <typename T>
hipError_t dalloc(T** p, size_t n) {
    return hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T) > 0 ? n * sizeof(T) : 16);
}
}  // namespace

struct he_engine {
    int device = 0;
    he_sim_params params{};
    he_model model{};
    bool has_model = false;
    he_model* d_model = nullptr;
    PhysTopo* d_topo = nullptr;
    int num_envs = 0;
    float *root = nullptr, *dof_state = nullptr, *rb = nullptr, *cf = nullptr, *dof_force = nullptr, *targets = nullptr;
    int32_t* num_contacts = nullptr;
    int32_t* dropped = nullptr;
    float* cache = nullptr;
    float* init_root = nullptr;     // [N,13] HE_BUF_INIT_ROOT_STATE
    int32_t* meta_cache = nullptr;  // [N,8] the imitation kernel's per-env motion-metadata cache
    float* d_rest = nullptr;        // [24,3] zero-pose body origins in the root frame
    bool component_limits = false;  // a dof bound inside (-pi + guard, pi - guard): not implemented
    int fused_step = -1;            // he_env_step as one launch: 1 / 0 (he_set_fused_step), -1 auto
    const float *mass_scale = nullptr, *friction = nullptr;
    const int32_t* terrain_kind = nullptr;
    float *pd_offset = nullptr, *pd_scale = nullptr;
    int32_t* frozen = nullptr;
    int clip_actions = 1;
    bool has_pd = false;
    he_eval_buffers eval{};
    int has_eval = 0;
    he_amp_buffers amp{};
    int has_amp = 0;
    // motion library
    float *m_hot = nullptr, *m_cold = nullptr, *m_lengths = nullptr, *m_dt = nullptr;
    int64_t *m_starts = nullptr, *m_nframes = nullptr;
    int64_t m_frames = 0;
    int m_motions = 0;
    unsigned long long* stamps = nullptr;
    // the physics launch's dispatch order (he_kernels.h launch_physics_order), rebuilt from the envs'
    // cycle counts every order_every launches; HE_PHYS_ORDER=0 keeps workgroup id = env
    int32_t* order = nullptr;    // [N]
    uint32_t* cost = nullptr;    // [N]
    int order_every = 8;
    long long launches = 0;
    // HE_TGS_LEGS=0 in the environment: no leg class (physics_kernel_tgs's Zh products over every dof
    // for every env; the results are the same bits, tests/test_full_size.py checks it)
    int full_dofs = 0;
    // the order rebuild runs on the launch's stream, and order_ready is recorded behind it: a physics
    // launch on another stream waits for it, so no workgroup reads a half-written order (a rebuild
    // on a side stream, beside the imitation step, made both slower: r06 A/B)
    hipEvent_t order_ready = nullptr;
    long long order_seq = 0;          // rebuilds issued
    long long order_seen_seq = -1;    // the rebuild the last physics launch waited for, on ...
    hipStream_t order_seen_stream = nullptr;  // ... this stream
};

extern "C" {

const char* he_last_error(void) { return g_err.c_str(); }
int he_version(void) { return 1; }

int he_device_count(int* count) {
    HE_CHECK(hipGetDeviceCount(count));
    return 0;
}

int he_create(const he_sim_params* params, int device, he_engine** out) {
    if (!params || !out) return fail("he_create: null argument");
    int n = 0;
    HE_CHECK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail("he_create: device %d out of range (%d devices)", device, n);
    hipDeviceProp_t prop;
    HE_CHECK(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail("he_create: device %d is %s; this build targets gfx950 (MI355X)", device, prop.gcnArchName);
    if (params->max_contacts < 1 || params->max_contacts > HE_MAX_CONTACTS)
        return fail("he_create: max_contacts must be in [1, %d]", HE_MAX_CONTACTS);
    if (params->dt <= 0.f) return fail("he_create: dt must be positive");
    if (params->substeps < 1 || params->substeps > 16) return fail("he_create: substeps must be in [1, 16]");
    if (!(params->max_joint_velocity > 0.f) || !(params->max_angular_velocity > 0.f))
        return fail("he_create: max_joint_velocity and max_angular_velocity must be positive");
    // sim_params.physx.solver_type (isaacgym_env.py:16): 0 PGS, 1 TGS with solver_iterations position
    // iterations (num_position_iterations, :17) per physics step
    if (params->solver_type != 0 && params->solver_type != 1)
        return fail("he_create: solver_type must be 0 (PGS) or 1 (TGS), got %d", params->solver_type);
    if (params->solver_type == 1 && (params->solver_iterations < 1 || params->solver_iterations > 16))
        return fail("he_create: TGS needs solver_iterations (position iterations) in [1, 16]");
    he_engine* h = new he_engine();
    h->device = device;
    h->params = *params;
    *out = h;
    return 0;
}

int he_set_model(he_engine* h, const he_model* model) {
    if (!h || !model) return fail("he_set_model: null argument");
    if (model->num_bodies != HE_NUM_BODIES || model->num_dof != HE_NUM_DOF)
        return fail("he_set_model: engine is built for %d bodies / %d dofs (got %d / %d)", HE_NUM_BODIES, HE_NUM_DOF,
                    model->num_bodies, model->num_dof);
    if (model->num_pairs < 0 || model->num_pairs > HE_MAX_PAIRS) return fail("he_set_model: bad pair count");
    if (model->parents[0] != -1) return fail("he_set_model: body 0 must be the root");
    for (int b = 1; b < HE_NUM_BODIES; ++b)
        if (model->parents[b] < 0 || model->parents[b] >= b) return fail("he_set_model: bodies must be in DFS order");
    for (int b = 0; b < HE_NUM_BODIES; ++b)
        if (model->geom_type[b] != HE_GEOM_SPHERE && model->geom_type[b] != HE_GEOM_CAPSULE && model->geom_type[b] != HE_GEOM_BOX)
            return fail("he_set_model: body %d has geom type %d (sphere 0, capsule 1, box 2)", b, model->geom_type[b]);
    // every check before the engine changes: a refused model leaves the previous one in place
    PhysTopo topo{};
    he_build_topo(*model, topo);
    if (topo.nnz > HE_NNZ_MAX) return fail("he_set_model: mass-matrix pattern too large (%d)", topo.nnz);
    if (topo.num_boxes > HE_MAX_BOXES)
        return fail("he_set_model: %d box geoms (the kernel's corner lanes hold at most %d)", topo.num_boxes, HE_MAX_BOXES);
    HE_CHECK(hipSetDevice(h->device));
    h->model = *model;
    // the kernel holds every joint's rotation angle below pi - 0.02 (the exp-map branch cut); dof
    // bounds inside that band would need per-component rows (the oracle has them, the kernel not)
    h->component_limits = false;
    for (int d = 0; d < HE_NUM_DOF; ++d)
        if (std::fabs(model->dof_lower[d]) < 3.1215f || std::fabs(model->dof_upper[d]) < 3.1215f) h->component_limits = true;
    if (!h->d_model) HE_CHECK(dalloc(&h->d_model, 1));
    if (!h->d_topo) HE_CHECK(dalloc(&h->d_topo, 1));
    HE_CHECK(hipMemcpy(h->d_model, model, sizeof(he_model), hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(h->d_topo, &topo, sizeof(PhysTopo), hipMemcpyHostToDevice));
    // the zero pose's body origins in the root frame: every local rotation is the identity, so the
    // joint offsets add up along the chain (the Default state init's rigid-body rows)
    float rest[HE_NUM_BODIES][3] = {};
    for (int b = 1; b < HE_NUM_BODIES; ++b)
        for (int c = 0; c < 3; ++c) rest[b][c] = rest[model->parents[b]][c] + model->local_pos[b][c];
    if (!h->d_rest) HE_CHECK(dalloc(&h->d_rest, HE_NUM_BODIES * 3));
    HE_CHECK(hipMemcpy(h->d_rest, rest, sizeof(rest), hipMemcpyHostToDevice));
    h->has_model = true;
    return 0;
}

static int warm_kernels(int device);

int he_create_envs(he_engine* h, int num_envs, const float* host_start_xy) {
    if (!h) return fail("he_create_envs: null handle");
    if (!h->has_model) return fail("he_create_envs: call he_set_model first");
    if (num_envs <= 0) return fail("he_create_envs: num_envs must be positive");
    if (h->num_envs) return fail("he_create_envs: envs already created");
    HE_CHECK(hipSetDevice(h->device));
    // before any allocation: a failed warm-up leaves nothing behind to leak or re-allocate
    if (warm_kernels(h->device)) return 1;
    const int N = num_envs;
    HE_CHECK(dalloc(&h->root, (size_t)N * 13));
    HE_CHECK(dalloc(&h->dof_state, (size_t)N * HE_NUM_DOF * 2));
    HE_CHECK(dalloc(&h->rb, (size_t)N * HE_NUM_BODIES * 13));
    HE_CHECK(dalloc(&h->cf, (size_t)N * HE_NUM_BODIES * 3));
    HE_CHECK(dalloc(&h->dof_force, (size_t)N * HE_NUM_DOF));
    HE_CHECK(dalloc(&h->targets, (size_t)N * HE_NUM_DOF));
    HE_CHECK(dalloc(&h->num_contacts, (size_t)N));
    HE_CHECK(dalloc(&h->dropped, (size_t)N));
    HE_CHECK(dalloc(&h->cache, (size_t)N * HE_CACHE_WORDS));
    // humanoid_phc.py:340-347: start pose (x, y) + z 0.89, identity rotation, zero velocity
    std::vector<float> root((size_t)N * 13, 0.f);
    for (int e = 0; e < N; ++e) {
        float* r = &root[(size_t)e * 13];
        r[0] = host_start_xy ? host_start_xy[2 * e] : 0.f;
        r[1] = host_start_xy ? host_start_xy[2 * e + 1] : 0.f;
        r[2] = 0.89f;
        r[6] = 1.f;
    }
    HE_CHECK(hipMemcpy(h->root, root.data(), root.size() * sizeof(float), hipMemcpyHostToDevice));
    // _initial_humanoid_root_states (humanoid_phc.py:522-523): the creation poses, zero velocities
    HE_CHECK(dalloc(&h->init_root, (size_t)N * 13));
    HE_CHECK(hipMemcpy(h->init_root, root.data(), root.size() * sizeof(float), hipMemcpyHostToDevice));
    HE_CHECK(hipMemset(h->dof_state, 0, (size_t)N * HE_NUM_DOF * 2 * sizeof(float)));
    HE_CHECK(hipMemset(h->rb, 0, (size_t)N * HE_NUM_BODIES * 13 * sizeof(float)));
    HE_CHECK(hipMemset(h->cf, 0, (size_t)N * HE_NUM_BODIES * 3 * sizeof(float)));
    HE_CHECK(hipMemset(h->dof_force, 0, (size_t)N * HE_NUM_DOF * sizeof(float)));
    HE_CHECK(hipMemset(h->targets, 0, (size_t)N * HE_NUM_DOF * sizeof(float)));
    HE_CHECK(hipMemset(h->num_contacts, 0, (size_t)N * sizeof(int32_t)));
    HE_CHECK(hipMemset(h->dropped, 0, (size_t)N * sizeof(int32_t)));
    HE_CHECK(hipMemset(h->cache, 0, (size_t)N * HE_CACHE_WORDS * sizeof(float)));
    HE_CHECK(dalloc(&h->meta_cache, (size_t)N * 8));
    HE_CHECK(hipMemset(h->meta_cache, 0xFF, (size_t)N * 8 * sizeof(int32_t)));  // motion -1: empty
    // dispatch order: the identity until the first rebuild
    std::vector<int32_t> ord((size_t)N);
    for (int e = 0; e < N; ++e) ord[e] = e;
    HE_CHECK(dalloc(&h->order, (size_t)N));
    HE_CHECK(hipMemcpy(h->order, ord.data(), ord.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    HE_CHECK(dalloc(&h->cost, (size_t)N));
    HE_CHECK(hipMemset(h->cost, 0, (size_t)N * sizeof(uint32_t)));
    if (const char* v = std::getenv("HE_PHYS_ORDER")) h->order_every = std::atoi(v);
    if (const char* v = std::getenv("HE_TGS_LEGS")) h->full_dofs = std::atoi(v) == 0;
    h->num_envs = N;
    return 0;
}

int he_destroy(he_engine* h) {
    if (!h) return 0;
    hipSetDevice(h->device);
    void* ptrs[] = {h->d_model, h->d_topo, h->root, h->dof_state, h->rb, h->cf, h->dof_force, h->targets,
                    h->num_contacts, h->dropped, h->cache, h->init_root, h->meta_cache, h->d_rest, h->pd_offset, h->pd_scale, h->frozen, h->m_hot, h->m_cold, h->m_lengths,
                    h->m_dt, h->m_starts, h->m_nframes, h->order, h->cost};
    for (void* p : ptrs)
        if (p) hipFree(p);
    if (h->order_ready) hipEventDestroy(h->order_ready);
    delete h;
    return 0;
}

int he_get_buffer(he_engine* h, int kind, void** dptr, int64_t* shape, int* ndim, int* dtype) {
    if (!h || !dptr || !shape || !ndim || !dtype) return fail("he_get_buffer: null argument");
    if (!h->num_envs) return fail("he_get_buffer: no envs created");
    const int64_t N = h->num_envs;
    *dtype = HE_DTYPE_F32;
    switch (kind) {
        case HE_BUF_ROOT_STATE: *dptr = h->root; *ndim = 2; shape[0] = N; shape[1] = 13; break;
        case HE_BUF_DOF_STATE: *dptr = h->dof_state; *ndim = 2; shape[0] = N * HE_NUM_DOF; shape[1] = 2; break;
        case HE_BUF_RB_STATE: *dptr = h->rb; *ndim = 2; shape[0] = N * HE_NUM_BODIES; shape[1] = 13; break;
        case HE_BUF_CONTACT_FORCE: *dptr = h->cf; *ndim = 2; shape[0] = N * HE_NUM_BODIES; shape[1] = 3; break;
        case HE_BUF_DOF_FORCE: *dptr = h->dof_force; *ndim = 1; shape[0] = N * HE_NUM_DOF; break;
        case HE_BUF_DOF_TARGET: *dptr = h->targets; *ndim = 2; shape[0] = N; shape[1] = HE_NUM_DOF; break;
        case HE_BUF_NUM_CONTACTS: *dptr = h->num_contacts; *ndim = 1; shape[0] = N; *dtype = HE_DTYPE_I32; break;
        case HE_BUF_DROPPED_CONTACTS: *dptr = h->dropped; *ndim = 1; shape[0] = N; *dtype = HE_DTYPE_I32; break;
        case HE_BUF_CONTACT_CACHE: *dptr = h->cache; *ndim = 2; shape[0] = N; shape[1] = HE_CACHE_WORDS; break;
        case HE_BUF_INIT_ROOT_STATE: *dptr = h->init_root; *ndim = 2; shape[0] = N; shape[1] = 13; break;
        case HE_BUF_PHYS_ORDER: *dptr = h->order; *ndim = 1; shape[0] = N; *dtype = HE_DTYPE_I32; break;
        case HE_BUF_PHYS_COST: *dptr = h->cost; *ndim = 1; shape[0] = N; *dtype = HE_DTYPE_I32; break;
        default: return fail("he_get_buffer: unknown buffer kind %d", kind);
    }
    return 0;
}

int he_set_dof_targets(he_engine* h, const float* src, void* stream) {
    if (!h || !src) return fail("he_set_dof_targets: null argument");
    if (src == h->targets) return 0;
    HE_CHECK(hipMemcpyAsync(h->targets, src, (size_t)h->num_envs * HE_NUM_DOF * sizeof(float),
                            hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return 0;
}

namespace {
static __global__ void copy_rows_kernel(float* dst, const float* src, const int32_t* ids, int k, int row, int num_rows) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= k * row) return;
    int i = t / row, c = t - i * row;
    int id = ids[i];
    if (id < 0 || id >= num_rows) return;
    dst[(size_t)id * row + c] = src[(size_t)id * row + c];
}

static int copy_rows(float* dst, const float* src, const int32_t* ids, int k, int row, int num_rows, void* stream,
              const char* what) {
    if (!src || !ids) return fail("%s: null argument", what);
    if (k < 0) return fail("%s: negative count", what);
    if (k == 0 || src == dst) return 0;
    int total = k * row;
    copy_rows_kernel<<<(total + 255) / 256, 256, 0, (hipStream_t)stream>>>(dst, src, ids, k, row, num_rows);
    HE_CHECK(hipGetLastError());
    return 0;
}
}  // namespace

// The env step's kernels (physics, imitation, motion ingestion, indexed row copies) each pay a
// one-time first-dispatch cost (~0.4-0.8 ms per kernel on the MI355X; 16-30 ms under rocprofv3's
// kernel tracing), paid here once per process and device at env creation, instead of by the setup's
// first full reset or by a timed step (he_kernels.h: warm_*_kernels). The rollout handoff kernels
// (he_rollout.hip, include/humanoid_rollout.h) are not on the env step and are not warmed: they pay
// theirs at the first Experience store. Serialised by a mutex (engines may be created from several
// threads); a failed warm-up is not recorded, so the next he_create_envs retries it.
static int warm_kernels(int device) {
    static std::mutex mu;
    static bool warmed[64] = {};
    const int wm = std::getenv("HE_WARM_MODE") ? std::atoi(std::getenv("HE_WARM_MODE")) : 2;
    if (wm <= 0 || device < 0 || device >= 64) return 0;
    std::lock_guard<std::mutex> lock(mu);
    if (warmed[device]) return 0;
    if (wm == 2) {
        copy_rows_kernel<<<1, 256>>>(nullptr, nullptr, nullptr, 0, 1, 0);
        HE_CHECK(hipGetLastError());
    }
    HE_CHECK(warm_physics_kernels(nullptr, wm));
    HE_CHECK(warm_imitation_kernels(nullptr, wm));
    HE_CHECK(warm_ingest_kernels(nullptr, wm));
    HE_CHECK(hipDeviceSynchronize());
    warmed[device] = true;
    return 0;
}

int he_set_root_state_indexed(he_engine* h, const float* src, const int32_t* ids, int k, void* stream) {
    if (!h) return fail("he_set_root_state_indexed: null handle");
    return copy_rows(h->root, src, ids, k, 13, h->num_envs, stream, "he_set_root_state_indexed");
}
int he_set_dof_state_indexed(he_engine* h, const float* src, const int32_t* ids, int k, void* stream) {
    if (!h) return fail("he_set_dof_state_indexed: null handle");
    return copy_rows(h->dof_state, src, ids, k, HE_NUM_DOF * 2, h->num_envs, stream, "he_set_dof_state_indexed");
}
int he_set_dof_targets_indexed(he_engine* h, const float* src, const int32_t* ids, int k, void* stream) {
    if (!h) return fail("he_set_dof_targets_indexed: null handle");
    return copy_rows(h->targets, src, ids, k, HE_NUM_DOF, h->num_envs, stream, "he_set_dof_targets_indexed");
}

int he_set_env_properties(he_engine* h, const float* mass_scale, const float* friction, const int32_t* terrain_kind) {
    if (!h) return fail("he_set_env_properties: null handle");
    h->mass_scale = mass_scale;
    h->friction = friction;
    h->terrain_kind = terrain_kind;
    h->params.terrain = terrain_kind ? 1 : 0;
    return 0;
}

int he_set_pd_params(he_engine* h, const float* host_offset, const float* host_scale, const int32_t* host_frozen_mask,
                     int clip_actions) {
    if (!h || !host_offset || !host_scale) return fail("he_set_pd_params: null argument");
    HE_CHECK(hipSetDevice(h->device));
    if (!h->pd_offset) HE_CHECK(dalloc(&h->pd_offset, HE_NUM_DOF));
    if (!h->pd_scale) HE_CHECK(dalloc(&h->pd_scale, HE_NUM_DOF));
    if (!h->frozen) HE_CHECK(dalloc(&h->frozen, HE_NUM_DOF));
    std::vector<int32_t> fz(HE_NUM_DOF, 0);
    if (host_frozen_mask) std::memcpy(fz.data(), host_frozen_mask, sizeof(int32_t) * HE_NUM_DOF);
    HE_CHECK(hipMemcpy(h->pd_offset, host_offset, sizeof(float) * HE_NUM_DOF, hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(h->pd_scale, host_scale, sizeof(float) * HE_NUM_DOF, hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(h->frozen, fz.data(), sizeof(int32_t) * HE_NUM_DOF, hipMemcpyHostToDevice));
    h->clip_actions = clip_actions;
    h->has_pd = true;
    return 0;
}

namespace {
// num_simulate gym.simulate() calls = num_simulate x SimParams.substeps physics steps of dt / substeps
static PhysArgs phys_args(he_engine* h, int num_simulate, const float* actions) {
    PhysArgs a{};
    a.p = h->params;
    a.p.dt = h->params.dt / (float)h->params.substeps;
    a.model = h->d_model;
    a.topo = h->d_topo;
    a.root_states = h->root;
    a.dof_state = h->dof_state;
    a.dof_targets = h->targets;
    a.actions = actions;
    a.pd_offset = h->pd_offset;
    a.pd_scale = h->pd_scale;
    a.frozen = h->frozen;
    a.clip_actions = h->clip_actions;
    a.rb_state = h->rb;
    a.contact_forces = h->cf;
    a.dof_force = h->dof_force;
    a.num_contacts = h->num_contacts;
    a.dropped = h->dropped;
    a.cache = h->cache;
    a.mass_scale = h->mass_scale;
    a.friction = h->friction;
    a.terrain_kind = h->terrain_kind;
    a.num_envs = h->num_envs;
    a.substeps = num_simulate * h->params.substeps;
    a.stamps = h->stamps;
    const bool ordered = h->order_every > 0;
    a.order = ordered ? h->order : nullptr;
    a.cost = ordered ? h->cost : nullptr;
    a.full_dofs = h->full_dofs;
    return a;
}
}  // namespace

// the physics launch, then every order_every launches the next launches' dispatch order from this
// one's per-env cycles (heavy envs first, he_kernels.h launch_physics_order)
static int physics_and_order(he_engine* h, const PhysArgs& a, hipStream_t stream) {
    if (a.order && h->order_seq > 0 && (h->order_seen_seq != h->order_seq || h->order_seen_stream != stream)) {
        HE_CHECK(hipStreamWaitEvent(stream, h->order_ready, 0));
        h->order_seen_seq = h->order_seq;
        h->order_seen_stream = stream;
    }
    HE_CHECK(launch_physics(a, stream));
    if (a.order && ++h->launches % h->order_every == 0) {
        if (!h->order_ready) HE_CHECK(hipEventCreateWithFlags(&h->order_ready, hipEventDisableTiming));
        HE_CHECK(launch_physics_order(h->cost, h->order, h->num_envs, stream));
        HE_CHECK(hipEventRecord(h->order_ready, stream));
        h->order_seen_seq = ++h->order_seq;
        h->order_seen_stream = stream;
    }
    return 0;
}

int he_simulate(he_engine* h, int num_simulate, void* stream) {
    if (!h || !h->num_envs) return fail("he_simulate: no envs");
    if (h->params.joint_limits && h->component_limits)
        return fail("he_simulate: dof ranges inside +-(pi - 0.02) need per-component limit rows (not implemented)");
    if (num_simulate < 1) return fail("he_simulate: num_simulate must be >= 1");
    if (physics_and_order(h, phys_args(h, num_simulate, nullptr), (hipStream_t)stream)) return 1;
    return 0;
}

int he_step_actions(he_engine* h, const float* actions, int num_simulate, void* stream) {
    if (!h || !h->num_envs || !actions) return fail("he_step_actions: bad arguments");
    if (!h->has_pd) return fail("he_step_actions: call he_set_pd_params first");
    if (h->params.joint_limits && h->component_limits)
        return fail("he_step_actions: dof ranges inside +-(pi - 0.02) need per-component limit rows (not implemented)");
    if (num_simulate < 1) return fail("he_step_actions: num_simulate must be >= 1");
    if (physics_and_order(h, phys_args(h, num_simulate, actions), (hipStream_t)stream)) return 1;
    return 0;
}

int he_refresh(he_engine* h, void* stream) {
    (void)stream;
    if (!h) return fail("he_refresh: null handle");
    return 0;
}

// new motion tables: the imitation kernel's per-env metadata cache (keyed by motion id) is stale
static hipError_t invalidate_meta_cache(he_engine* h) {
    if (!h->meta_cache) return hipSuccess;
    return hipMemset(h->meta_cache, 0xFF, (size_t)h->num_envs * 8 * sizeof(int32_t));
}

int he_load_motions(he_engine* h, int64_t F, int M, const float* gts, const float* grs, const float* lrs,
                    const float* gvs, const float* gavs, const float* dvs, const int64_t* length_starts,
                    const int64_t* num_frames, const float* lengths, const float* dt) {
    if (!h) return fail("he_load_motions: null handle");
    if (F <= 0 || M <= 0 || !gts || !grs || !lrs || !gvs || !gavs || !dvs || !length_starts || !num_frames ||
        !lengths || !dt)
        return fail("he_load_motions: bad arguments");
    for (int i = 0; i < M; ++i) {
        if (num_frames[i] < 1 || length_starts[i] < 0 || length_starts[i] + num_frames[i] > F)
            return fail("he_load_motions: motion %d frames [%lld, +%lld) outside the %lld-frame table", i,
                        (long long)length_starts[i], (long long)num_frames[i], (long long)F);
    }
    HE_CHECK(hipSetDevice(h->device));
    const int B = HE_NUM_BODIES;
    std::vector<float> hot((size_t)F * B * HE_MOTION_HOT), cold((size_t)F * B * HE_MOTION_COLD, 0.f);
    for (int64_t f = 0; f < F; ++f)
        for (int b = 0; b < B; ++b) {
            float* r = &hot[((size_t)f * B + b) * HE_MOTION_HOT];
            const size_t i3 = ((size_t)f * B + b) * 3, i4 = ((size_t)f * B + b) * 4;
            r[0] = gts[i3]; r[1] = gts[i3 + 1]; r[2] = gts[i3 + 2];
            r[3] = grs[i4]; r[4] = grs[i4 + 1]; r[5] = grs[i4 + 2]; r[6] = grs[i4 + 3];
            r[7] = gvs[i3]; r[8] = gvs[i3 + 1]; r[9] = gvs[i3 + 2];
            r[10] = gavs[i3]; r[11] = gavs[i3 + 1]; r[12] = gavs[i3 + 2];
            float* c = &cold[((size_t)f * B + b) * HE_MOTION_COLD];
            c[0] = lrs[i4]; c[1] = lrs[i4 + 1]; c[2] = lrs[i4 + 2]; c[3] = lrs[i4 + 3];
            if (b > 0) {
                const size_t d3 = ((size_t)f * (B - 1) + b - 1) * 3;
                c[4] = dvs[d3]; c[5] = dvs[d3 + 1]; c[6] = dvs[d3 + 2];
            }
        }
    void* old[] = {h->m_hot, h->m_cold, h->m_lengths, h->m_dt, h->m_starts, h->m_nframes};
    for (void* p : old)
        if (p) HE_CHECK(hipFree(p));
    HE_CHECK(dalloc(&h->m_hot, hot.size()));
    HE_CHECK(dalloc(&h->m_cold, cold.size()));
    HE_CHECK(dalloc(&h->m_lengths, (size_t)M));
    HE_CHECK(dalloc(&h->m_dt, (size_t)M));
    HE_CHECK(dalloc(&h->m_starts, (size_t)M));
    HE_CHECK(dalloc(&h->m_nframes, (size_t)M));
    HE_CHECK(hipMemcpy(h->m_hot, hot.data(), hot.size() * sizeof(float), hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(h->m_cold, cold.data(), cold.size() * sizeof(float), hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(h->m_lengths, lengths, M * sizeof(float), hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(h->m_dt, dt, M * sizeof(float), hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(h->m_starts, length_starts, M * sizeof(int64_t), hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(h->m_nframes, num_frames, M * sizeof(int64_t), hipMemcpyHostToDevice));
    h->m_frames = F;
    h->m_motions = M;
    HE_CHECK(invalidate_meta_cache(h));
    return 0;
}

int he_ingest_clips(he_engine* h, int num_clips, const int64_t* host_num_frames, const float* host_fps,
                    const float* pose_quat_global, const float* root_trans, int num_motions,
                    const int32_t* host_motion_clip, void* stream) {
    if (!h) return fail("he_ingest_clips: null handle");
    if (!h->has_model) return fail("he_ingest_clips: call he_set_model first");
    if (num_clips <= 0 || !host_num_frames || !host_fps || !pose_quat_global || !root_trans)
        return fail("he_ingest_clips: bad arguments");
    if (num_motions <= 0) num_motions = num_clips;
    if (!host_motion_clip && num_motions != num_clips)
        return fail("he_ingest_clips: motion->clip map required when num_motions != num_clips");
    std::vector<int64_t> cstart(num_clips), cnf(num_clips);
    std::vector<float> cdt(num_clips);
    int64_t F = 0;
    for (int c = 0; c < num_clips; ++c) {
        if (host_num_frames[c] < 1 || !(host_fps[c] > 0.f))
            return fail("he_ingest_clips: clip %d has %lld frames at %g fps", c, (long long)host_num_frames[c],
                        (double)host_fps[c]);
        cstart[c] = F;
        cnf[c] = host_num_frames[c];
        cdt[c] = (float)(1.0 / (double)host_fps[c]);
        F += host_num_frames[c];
    }
    std::vector<int64_t> ms(num_motions), mn(num_motions);
    std::vector<float> ml(num_motions), mdt(num_motions);
    for (int i = 0; i < num_motions; ++i) {
        const int c = host_motion_clip ? host_motion_clip[i] : i;
        if (c < 0 || c >= num_clips) return fail("he_ingest_clips: motion %d maps to clip %d of %d", i, c, num_clips);
        ms[i] = cstart[c];
        mn[i] = cnf[c];
        // motion_lib.py:376-379: curr_len = 1/fps * (num_frames - 1) in python floats -> float32
        ml[i] = (float)(1.0 / (double)host_fps[c] * (double)(cnf[c] - 1));
        mdt[i] = (float)(1.0 / (double)host_fps[c]);
    }
    HE_CHECK(hipSetDevice(h->device));
    const hipStream_t st = (hipStream_t)stream;
    HE_CHECK(hipStreamSynchronize(st));  // tables may be in use by queued kernels
    void* old[] = {h->m_hot, h->m_cold, h->m_lengths, h->m_dt, h->m_starts, h->m_nframes};
    for (void* p : old)
        if (p) HE_CHECK(hipFree(p));
    h->m_hot = h->m_cold = h->m_lengths = h->m_dt = nullptr;
    h->m_starts = h->m_nframes = nullptr;
    h->m_motions = 0;
    const int B = HE_NUM_BODIES;
    HE_CHECK(dalloc(&h->m_hot, (size_t)F * B * HE_MOTION_HOT));
    HE_CHECK(dalloc(&h->m_cold, (size_t)F * B * HE_MOTION_COLD));
    HE_CHECK(dalloc(&h->m_lengths, (size_t)num_motions));
    HE_CHECK(dalloc(&h->m_dt, (size_t)num_motions));
    HE_CHECK(dalloc(&h->m_starts, (size_t)num_motions));
    HE_CHECK(dalloc(&h->m_nframes, (size_t)num_motions));
    HE_CHECK(hipMemcpy(h->m_lengths, ml.data(), num_motions * sizeof(float), hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(h->m_dt, mdt.data(), num_motions * sizeof(float), hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(h->m_starts, ms.data(), num_motions * sizeof(int64_t), hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(h->m_nframes, mn.data(), num_motions * sizeof(int64_t), hipMemcpyHostToDevice));
    int64_t *d_cs = nullptr, *d_cn = nullptr;
    float *d_cdt = nullptr, *scratch = nullptr;
    HE_CHECK(dalloc(&d_cs, (size_t)num_clips));
    HE_CHECK(dalloc(&d_cn, (size_t)num_clips));
    HE_CHECK(dalloc(&d_cdt, (size_t)num_clips));
    HE_CHECK(dalloc(&scratch, (size_t)F * B * 3));
    HE_CHECK(hipMemcpy(d_cs, cstart.data(), num_clips * sizeof(int64_t), hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(d_cn, cnf.data(), num_clips * sizeof(int64_t), hipMemcpyHostToDevice));
    HE_CHECK(hipMemcpy(d_cdt, cdt.data(), num_clips * sizeof(float), hipMemcpyHostToDevice));
    hipError_t e = launch_ingest(pose_quat_global, root_trans, h->d_model->parents, &h->d_model->local_pos[0][0],
                                 d_cs, d_cn, d_cdt, num_clips, F, h->m_hot, h->m_cold, scratch, st);
    hipError_t e2 = hipStreamSynchronize(st);
    hipFree(d_cs); hipFree(d_cn); hipFree(d_cdt); hipFree(scratch);
    HE_CHECK(e);
    HE_CHECK(e2);
    h->m_frames = F;
    h->m_motions = num_motions;
    HE_CHECK(invalidate_meta_cache(h));
    return 0;
}

namespace {
static MotionDev motion_dev(he_engine* h) {
    return MotionDev{h->m_hot, h->m_cold, h->m_starts, h->m_nframes, h->m_lengths, h->m_dt, h->m_motions};
}

static int imit_common(he_engine* h, const he_imitation_params* p, const he_env_motion* em, ImitArgs& a, const char* what) {
    if (!h || !p || !em) return fail("%s: null argument", what);
    if (!h->num_envs) return fail("%s: no envs", what);
    if (!h->m_motions) return fail("%s: call he_load_motions first", what);
    if (!em->motion_ids || !em->start_times || !em->start_offsets || !em->global_offset || !em->progress)
        return fail("%s: he_env_motion has null buffers", what);
    a = ImitArgs{};
    a.p = *p;
    a.m = motion_dev(h);
    a.root_states = h->root;
    a.dof_state = h->dof_state;
    a.rb_state = h->rb;
    a.contact_forces = h->cf;
    a.dof_force = h->dof_force;
    a.dof_targets = h->targets;
    a.motion_ids = em->motion_ids;
    a.start_times = em->start_times;
    a.start_offsets = em->start_offsets;
    a.global_offset = em->global_offset;
    a.progress = em->progress;
    a.ev = h->eval;
    a.has_eval = h->has_eval;
    a.init_root = h->init_root;
    a.rest_pos = h->d_rest;
    a.meta_cache = h->meta_cache;
    if (p->state_init < HE_STATE_INIT_DEFAULT || p->state_init > HE_STATE_INIT_HYBRID)
        return fail("%s: state_init %d is not a StateInit (0 Default, 1 Start, 2 Random, 3 Hybrid)", what, p->state_init);
    if (p->state_init == HE_STATE_INIT_HYBRID && !(p->hybrid_init_prob >= 0.f && p->hybrid_init_prob <= 1.f))
        return fail("%s: hybrid_init_prob must be in [0, 1]", what);
    return 0;
}
// the AMP update that follows an imitation launch (he_set_amp)
static hipError_t amp_after(he_engine* h, const ImitArgs& ia, int mode, hipStream_t stream) {
    if (!h->has_amp) return hipSuccess;
    AmpArgs a{};
    a.m = ia.m;
    a.rb_state = h->rb;
    a.dof_state = h->dof_state;
    a.motion_ids = ia.motion_ids;
    a.start_times = ia.start_times;
    a.reset = ia.reset;
    a.env_ids = ia.env_ids;
    a.count = ia.count;
    a.mode = mode;
    a.control_dt = ia.p.control_dt;
    a.amp = h->amp;
    a.ip = ia.p;
    a.phases = ia.phases;
    a.seed = ia.seed;
    a.step = ia.step;
    return launch_amp(a, stream);
}
}  // namespace

int he_imitation_step(he_engine* h, const he_imitation_params* p, const he_env_motion* em, float* obs, float* rew,
                      float* reward_raw, uint8_t* reset, uint8_t* terminate, void* stream) {
    ImitArgs a;
    if (imit_common(h, p, em, a, "he_imitation_step")) return 1;
    if (!obs || !rew || !reward_raw || !reset || !terminate) return fail("he_imitation_step: null output");
    a.obs = obs; a.rew = rew; a.reward_raw = reward_raw; a.reset = reset; a.terminate = terminate;
    a.count = h->num_envs;
    a.mode = 0;
    HE_CHECK(launch_imitation(a, (hipStream_t)stream));
    HE_CHECK(amp_after(h, a, 0, (hipStream_t)stream));
    return 0;
}

int he_set_eval(he_engine* h, const he_eval_buffers* b) {
    if (!h) return fail("he_set_eval: null engine");
    if (!b) {
        h->has_eval = 0;
        return 0;
    }
    if (!b->num_steps || !b->history || !b->sums) return fail("he_set_eval: num_steps, history and sums are required");
    if (b->frame < 0) return fail("he_set_eval: negative frame");
    h->eval = *b;
    h->has_eval = 1;
    return 0;
}

int he_reset_envs(he_engine* h, const he_imitation_params* p, const he_env_motion* em, const int32_t* env_ids, int k,
                  const float* phases, float* obs, uint8_t* reset, uint8_t* terminate, void* stream) {
    ImitArgs a;
    if (imit_common(h, p, em, a, "he_reset_envs")) return 1;
    if (k < 0) return fail("he_reset_envs: negative count");
    if (k == 0) return 0;
    if (!env_ids || !phases || !obs || !reset || !terminate) return fail("he_reset_envs: null argument");
    a.obs = obs; a.reset = reset; a.terminate = terminate;
    a.env_ids = env_ids;
    a.count = k;
    a.phases = phases;
    a.mode = 2;
    HE_CHECK(launch_imitation(a, (hipStream_t)stream));
    HE_CHECK(amp_after(h, a, 2, (hipStream_t)stream));
    return 0;
}

int he_env_step(he_engine* h, const he_imitation_params* p, const he_env_motion* em, const float* actions,
                int num_simulate, uint64_t seed, uint64_t step_index, float* obs, float* rew, float* reward_raw,
                uint8_t* reset, uint8_t* terminate, void* stream) {
    if (!h || !h->num_envs || !actions) return fail("he_env_step: bad arguments");
    // auto: one launch while the envs fit one round of waves on the chip (2 per SIMD: launch and
    // tail latency dominate there); past it two launches, because the imitation step at one env
    // per 250-VGPR wave adds more than the stand-alone kernel costs at full occupancy (r02 A/B at
    // 4096 envs: 0.218 against 0.209 ms per step)
    const bool fused = h->fused_step == 1 || (h->fused_step < 0 && h->num_envs <= 2048);
    if (h->has_eval || !fused) {  // eval recording lives in the stand-alone imitation kernel
        if (he_step_actions(h, actions, num_simulate, stream)) return 1;
        return he_imitation_reset_step(h, p, em, seed, step_index, obs, rew, reward_raw, reset, terminate, stream);
    }
    // one launch: actions -> PD targets -> physics -> the imitation step with the device reset of
    // flagged envs in the physics kernel's epilogue (the same results as the two launches)
    if (!h->has_pd) return fail("he_env_step: call he_set_pd_params first");
    if (num_simulate < 1) return fail("he_env_step: num_simulate must be >= 1");
    if (h->params.joint_limits && h->component_limits)
        return fail("he_env_step: dof ranges inside +-(pi - 0.02) need per-component limit rows (not implemented)");
    ImitArgs a;
    if (imit_common(h, p, em, a, "he_env_step")) return 1;
    if (!obs || !rew || !reward_raw || !reset || !terminate) return fail("he_env_step: null output");
    a.obs = obs; a.rew = rew; a.reward_raw = reward_raw; a.reset = reset; a.terminate = terminate;
    a.count = h->num_envs;
    a.mode = 1;
    a.seed = seed;
    a.step = step_index;
    PhysArgs pa = phys_args(h, num_simulate, actions);
    pa.fused = 1;
    pa.im = a;
    // with the heavy-first dispatch order as the two-launch form (the epilogue indexes the ordered
    // env): bit-identical to the unordered launch; at 4096 envs configs[4] 5 % faster, configs[1] / [2]
    // within 0.3 % (profiles/r05/ab_fused_order.txt)
    if (physics_and_order(h, pa, (hipStream_t)stream)) return 1;
    HE_CHECK(amp_after(h, a, 1, (hipStream_t)stream));
    return 0;
}

int he_set_fused_step(he_engine* h, int enable) {
    if (!h) return fail("he_set_fused_step: null engine");
    h->fused_step = enable < 0 ? -1 : (enable != 0);
    return 0;
}

int he_imitation_reset_step(he_engine* h, const he_imitation_params* p, const he_env_motion* em, uint64_t seed,
                            uint64_t step_index, float* obs, float* rew, float* reward_raw, uint8_t* reset,
                            uint8_t* terminate, void* stream) {
    ImitArgs a;
    if (imit_common(h, p, em, a, "he_imitation_reset_step")) return 1;
    if (!obs || !rew || !reward_raw || !reset || !terminate) return fail("he_imitation_reset_step: null output");
    a.obs = obs; a.rew = rew; a.reward_raw = reward_raw; a.reset = reset; a.terminate = terminate;
    a.count = h->num_envs;
    a.mode = 1;
    a.seed = seed;
    a.step = step_index;
    HE_CHECK(launch_imitation(a, (hipStream_t)stream));
    HE_CHECK(amp_after(h, a, 1, (hipStream_t)stream));
    return 0;
}

int he_set_amp(he_engine* h, const he_amp_buffers* b) {
    if (!h) return fail("he_set_amp: null engine");
    if (!b) {
        h->has_amp = 0;
        return 0;
    }
    if (!b->amp_obs) return fail("he_set_amp: amp_obs is required");
    if (b->num_steps < 1 || b->num_steps > HE_AMP_MAX_STEPS)
        return fail("he_set_amp: num_steps must be in [1, %d]", HE_AMP_MAX_STEPS);
    if ((reinterpret_cast<uintptr_t>(b->amp_obs) | reinterpret_cast<uintptr_t>(b->amp_obs_demo)) & 15)
        return fail("he_set_amp: buffers must be 16-byte aligned");
    h->amp = *b;
    h->has_amp = 1;
    return 0;
}

int he_amp_observations(int k, const float* root_pos, const float* root_rot, const float* root_vel,
                        const float* root_ang_vel, const float* dof_pos, const float* dof_vel,
                        const float* key_body_pos, float* out, void* stream) {
    if (k < 0) return fail("he_amp_observations: negative count");
    if (k == 0) return 0;
    if (!root_pos || !root_rot || !root_vel || !root_ang_vel || !dof_pos || !dof_vel || !key_body_pos || !out)
        return fail("he_amp_observations: null argument");
    AmpArgs a{};
    a.count = k;
    a.root_pos = root_pos; a.root_rot = root_rot; a.root_vel = root_vel; a.root_ang_vel = root_ang_vel;
    a.dof_pos = dof_pos; a.dof_vel = dof_vel; a.key_pos = key_body_pos; a.out = out;
    HE_CHECK(launch_amp_function(a, (hipStream_t)stream));
    return 0;
}

int he_motion_state(he_engine* h, int k, const int64_t* ids, const float* times, const float* offset, float* rg_pos,
                    float* rb_rot, float* body_vel, float* body_ang_vel, float* dof_pos, float* dof_vel, void* stream) {
    if (!h) return fail("he_motion_state: null handle");
    if (!h->m_motions) return fail("he_motion_state: call he_load_motions first");
    if (k < 0 || (k > 0 && (!ids || !times))) return fail("he_motion_state: bad arguments");
    MotionStateArgs a{};
    a.m = motion_dev(h);
    a.k = k;
    a.ids = ids;
    a.times = times;
    a.offset = offset;
    a.rg_pos = rg_pos; a.rb_rot = rb_rot; a.body_vel = body_vel; a.body_ang_vel = body_ang_vel;
    a.dof_pos = dof_pos; a.dof_vel = dof_vel;
    HE_CHECK(launch_motion_state(a, (hipStream_t)stream));
    return 0;
}

int he_set_debug_stamps(he_engine* h, uint64_t* device_buffer) {
    if (!h) return fail("he_set_debug_stamps: null handle");
    if (device_buffer && !physics_phase_stamps())
        return fail("he_set_debug_stamps: this library is built without phase stamps "
                    "(load libhumanoid_engine_phases.so, e.g. HE_ENGINE_LIB=humanoid_amd/libhumanoid_engine_phases.so)");
    h->stamps = reinterpret_cast<unsigned long long*>(device_buffer);
    return 0;
}

float he_hash_uniform(uint64_t seed, uint64_t step, uint32_t env) {
    uint64_t z = seed * 0x9E3779B97F4A7C15ull ^ (step + 0x632BE59BD9B4E019ull) * 0xBF58476D1CE4E5B9ull ^
                 ((uint64_t)env + 0x2545F4914F6CDD1Dull) * 0x94D049BB133111EBull;
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27; z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)(z >> 40) * (1.0f / 16777216.0f);
}

}  // extern "C"
