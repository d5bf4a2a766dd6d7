// he_rollout.hip -- rollout -> trainer handoff on the device, the C ABI of
// include/humanoid_rollout.h. Replaces, in puffer_phc/clean_pufferl/: Experience.store
// (structs.py:108-126), sort_training_data (:128-142), flatten_batch (:144-160), the Cython
// compute_gae (c_gae.pyx:11-32) and the advantage/return layout of train (core.py:213-256).
//
// Kernels (all HBM-bound byte movement except the GAE recurrence, which is latency-bound):
//   store_keys_kernel   per stored row: its flat destination (mask compaction = one block scan),
//                       env id and rank among that env's rows (atomic per-env counter);
//   rows_kernel         row copies, one wave per wide row (obs 934 f32 as float2), one lane per
//                       narrow row; STORE maps source row -> flat row, GATHER maps minibatch row ->
//                       sorted position -> flat row (the b_idxs transpose);
//   offsets_kernel +    counting sort by env id, stable in store order == Python's sorted() over
//   order_kernel        the (env_id, step) keys, since steps only grow with the store order;
//   gae_window_kernel   the GAE reverse recurrence, every position restarted W steps ahead (see
//                       gae_window below), operands staged in LDS;
//   gae_serial_kernel   the same recurrence run serially, for (gamma*lambda) too close to 1.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

#include "../../include/humanoid_rollout.h"
#include "he_kernels.h"

namespace {

constexpr int BLOCK = 256;
constexpr int WAVES = BLOCK / 64;

struct Fields {
    he_rollout_field f[HE_ROLLOUT_MAX_FIELDS];
};

// ---------------------------------------------------------------------------------------------
// store: destination rows and (env, rank) keys

struct StoreArgs {
    const int32_t* env_ids;
    const uint8_t* mask;     // null: every row
    int64_t rows, ptr, capacity;
    int32_t step, num_keys;
    int32_t *key_count, *key_last, *row_env, *row_rank, *scratch, *status;
};

__device__ void store_key(const StoreArgs& a, int64_t i, int64_t dst, int& err) {
    const int key = a.env_ids[i];
    if (key < 0 || key >= a.num_keys) {  // never index the per-env arrays with it
        err |= HE_ROLLOUT_ERR_KEY_RANGE;
        a.row_env[dst] = -1;
        a.row_rank[dst] = 0;
        return;
    }
    const int rank = atomicAdd(a.key_count + key, 1);
    if (atomicExch(a.key_last + key, a.step) == a.step) err |= HE_ROLLOUT_ERR_DUP_KEY;
    a.row_env[dst] = key;
    a.row_rank[dst] = rank;
}

// mask == null: row i -> ptr + i, any number of blocks
__global__ void __launch_bounds__(BLOCK) store_keys_dense_kernel(StoreArgs a) {
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    int err = 0;
    if (i < a.rows && a.ptr + i < a.capacity) store_key(a, i, a.ptr + i, err);
    if (err) atomicOr(a.status + 1, err);
    if (i == 0) a.status[0] = (int32_t)(a.rows < a.capacity - a.ptr ? a.rows : a.capacity - a.ptr);
}

// masked: one block compacts the selected rows in order (indices[: batch_size - ptr])
__global__ void __launch_bounds__(1024) store_keys_masked_kernel(StoreArgs a) {
    __shared__ int wave_tot[16];
    __shared__ int64_t base_s;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) base_s = 0;
    __syncthreads();
    int err = 0;
    for (int64_t c0 = 0; c0 < a.rows; c0 += 1024) {
        const int64_t i = c0 + threadIdx.x;
        const bool sel = i < a.rows && a.mask[i] != 0;
        const uint64_t bal = __ballot(sel);
        const int before = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wave_tot[wave] = __popcll(bal);
        __syncthreads();
        int off = 0, tot = 0;
        for (int w = 0; w < 16; ++w) {
            off += w < wave ? wave_tot[w] : 0;
            tot += wave_tot[w];
        }
        const int64_t dst = a.ptr + base_s + off + before;
        if (i < a.rows) {
            const bool keep = sel && dst < a.capacity;
            a.scratch[i] = keep ? (int32_t)dst : -1;
            if (keep) store_key(a, i, dst, err);
        }
        __syncthreads();
        if (threadIdx.x == 0) base_s += tot;
        __syncthreads();
    }
    if (err) atomicOr(a.status + 1, err);
    if (threadIdx.x == 0) {
        const int64_t room = a.capacity - a.ptr;
        a.status[0] = (int32_t)(base_s < room ? base_s : room);
    }
}

// ---------------------------------------------------------------------------------------------
// row copies

enum { MAP_STORE_DENSE = 0, MAP_STORE_MASKED = 1, MAP_GATHER = 2 };

struct RowsArgs {
    Fields fields;
    int64_t rows;            // STORE: source rows; GATHER: destination rows
    int64_t ptr, capacity;   // STORE
    const int32_t* scratch;  // STORE_MASKED
    const int64_t* idxs;     // GATHER
    int32_t num_mb, mb_rows, bptt;
    int mode;
};

// sorted position p of minibatch-ordered row d: d = (m*rows + r)*bptt + t, p = (r*num_mb + m)*bptt + t
__device__ __forceinline__ int64_t sorted_pos(int64_t d, int num_mb, int mb_rows, int bptt) {
    const int64_t per_mb = (int64_t)mb_rows * bptt;
    const int64_t m = d / per_mb, rem = d - m * per_mb;
    const int64_t r = rem / bptt, t = rem - r * bptt;
    return (r * num_mb + m) * bptt + t;
}

// (source row, destination row) of row index i, or src < 0 to skip
__device__ __forceinline__ void row_map(const RowsArgs& a, int64_t i, int64_t& src, int64_t& dst) {
    if (a.mode == MAP_GATHER) {
        dst = i;
        src = a.idxs[sorted_pos(i, a.num_mb, a.mb_rows, a.bptt)];
    } else {
        src = i;
        dst = a.mode == MAP_STORE_DENSE ? (a.ptr + i < a.capacity ? a.ptr + i : -1) : (int64_t)a.scratch[i];
        if (dst < 0) src = -1;
    }
}

__device__ __forceinline__ float load_elem(const he_rollout_field& f, int64_t k) {
    return f.src_kind == HE_ROLLOUT_U8 ? (static_cast<const uint8_t*>(f.src)[k] ? 1.0f : 0.0f)
                                       : static_cast<const float*>(f.src)[k];
}

// grid: x over rows (WAVES rows per block for wide fields, BLOCK rows for narrow), y = field
__global__ void __launch_bounds__(BLOCK) rows_kernel(RowsArgs a) {
    const he_rollout_field& f = a.fields.f[blockIdx.y];
    const int w = f.width;
    if (w >= 32) {  // one wave per row
        const int64_t i = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
        if (i >= a.rows) return;
        int64_t src, dst;
        row_map(a, i, src, dst);
        if (src < 0) return;
        const int lane = threadIdx.x & 63;
        float* d = f.dst + dst * w;
        if (f.src_kind == HE_ROLLOUT_F32 && (w & 1) == 0 &&
            ((reinterpret_cast<uintptr_t>(f.src) | reinterpret_cast<uintptr_t>(f.dst)) & 7) == 0) {
            const float2* s2 = reinterpret_cast<const float2*>(static_cast<const float*>(f.src) + src * w);
            float2* d2 = reinterpret_cast<float2*>(d);
            for (int c = lane; c < w / 2; c += 64) d2[c] = s2[c];
        } else {
            for (int c = lane; c < w; c += 64) d[c] = load_elem(f, src * w + c);
        }
    } else {  // one lane per row
        const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
        if (i >= a.rows) return;
        int64_t src, dst;
        row_map(a, i, src, dst);
        if (src < 0) return;
        for (int c = 0; c < w; ++c) f.dst[dst * w + c] = load_elem(f, src * w + c);
    }
}

int launch_rows(const RowsArgs& a, hipStream_t s, int num_fields) {
    if (a.rows <= 0 || num_fields <= 0) return 0;
    const int64_t gx = (a.rows + WAVES - 1) / WAVES;
    if (gx > 0x7fffffff) return he_fail_text("he_rollout: too many rows");
    rows_kernel<<<dim3((unsigned)gx, (unsigned)num_fields), BLOCK, 0, s>>>(a);
    return 0;
}

// ---------------------------------------------------------------------------------------------
// counting sort by env id

__global__ void __launch_bounds__(1024) offsets_kernel(const int32_t* count, int32_t* offset, int num_keys) {
    __shared__ int wave_tot[16];
    __shared__ int base_s;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) base_s = 0;
    __syncthreads();
    for (int c0 = 0; c0 < num_keys; c0 += 1024) {
        const int k = c0 + threadIdx.x;
        const int v = k < num_keys ? count[k] : 0;
        int incl = v;  // inclusive scan within the wave
        for (int d = 1; d < 64; d <<= 1) {
            const int o = __shfl_up(incl, d, 64);
            if (lane >= d) incl += o;
        }
        if (lane == 63) wave_tot[wave] = incl;
        __syncthreads();
        int off = 0, tot = 0;
        for (int w = 0; w < 16; ++w) {
            off += w < wave ? wave_tot[w] : 0;
            tot += wave_tot[w];
        }
        if (k < num_keys) offset[k] = base_s + off + incl - v;
        __syncthreads();
        if (threadIdx.x == 0) base_s += tot;
        __syncthreads();
    }
}

__global__ void __launch_bounds__(BLOCK) order_kernel(const int32_t* row_env, const int32_t* row_rank,
                                                      const int32_t* offset, int64_t rows, int64_t* idxs) {
    const int64_t r = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (r >= rows) return;
    const int key = row_env[r];
    if (key < 0) return;  // reported through the error bits
    const int64_t p = (int64_t)offset[key] + row_rank[r];
    if (p < rows) idxs[p] = r;
}

// ---------------------------------------------------------------------------------------------
// GAE. The Cython loop (c_gae.pyx:23-30), float32 throughout except `1.0 - done` (a C double):
//   adv[n-1] = 0; last = 0; for t = n-2 .. 0:
//     nnt = (float)(1.0 - done[t+1])
//     delta = (reward[t+1] + (gamma * value[t+1]) * nnt) - value[t]
//     last = delta + ((gamma * lambda) * nnt) * last;  adv[t] = last
// Position t depends on t+1.. only through `last`, whose weight shrinks by gamma*lambda per step:
// restarting the recurrence from last = 0 at t + W reproduces the serial float32 values: the two
// runs differ by (gamma*lambda)^k x |tail| in exact arithmetic, which falls below rounding after
// ~10 steps for the default gamma 0.98, lambda 0.2 (config.py:202-203); from the first step where
// both round to the same float they are identical. W is sized for (gamma*lambda)^W < 2^-200 (W = 78
// by default), which leaves ~65 steps of margin; a done at t' (nnt = 0) cuts the dependence
// exactly. The kernels spell every operation out (no contraction) so the rounding is the Cython
// module's; the GPU tests compare bit for bit.

struct GaeArgs {
    const float *dones, *values, *rewards, *extra;  // extra may be null
    const int64_t* idxs;                            // null: identity
    int64_t n;
    float gamma, lambda;
    int32_t window;
    int32_t num_mb, mb_rows, bptt;
    float *adv, *ret;  // ret may be null
};

__device__ __forceinline__ int64_t src_of(const GaeArgs& a, int64_t p) { return a.idxs ? a.idxs[p] : p; }

__device__ __forceinline__ int64_t dest_of(const GaeArgs& a, int64_t p) {
    if (a.num_mb == 1) return p;
    // inverse of sorted_pos: p = (r*num_mb + m)*bptt + t  ->  d = (m*mb_rows + r)*bptt + t
    const int64_t t = p % a.bptt, q = p / a.bptt;
    const int64_t m = q % a.num_mb, r = q / a.num_mb;
    return (m * a.mb_rows + r) * a.bptt + t;
}

__device__ __forceinline__ float gae_step(float last, float nnt, float v_next, float r_next, float v_cur, float g,
                                          float gl) {
    const float delta = __fsub_rn(__fadd_rn(r_next, __fmul_rn(__fmul_rn(g, v_next), nnt)), v_cur);
    return __fadd_rn(delta, __fmul_rn(__fmul_rn(gl, nnt), last));
}

__device__ __forceinline__ void gae_write(const GaeArgs& a, int64_t p, float adv, float v_cur) {
    const int64_t d = dest_of(a, p);
    a.adv[d] = adv;
    if (a.ret) a.ret[d] = __fadd_rn(adv, v_cur);
}

// block: BLOCK consecutive positions; LDS holds nnt / value / reward for [p0, p0 + BLOCK + W]
__global__ void __launch_bounds__(BLOCK) gae_window_kernel(GaeArgs a) {
    extern __shared__ float lds[];
    const int span = BLOCK + a.window + 1;
    float* s_nnt = lds;
    float* s_v = lds + span;
    float* s_r = lds + 2 * span;
    const int64_t p0 = (int64_t)blockIdx.x * BLOCK;
    for (int k = threadIdx.x; k < span; k += BLOCK) {
        const int64_t p = p0 + k;
        if (p < a.n) {
            const int64_t s = src_of(a, p);
            s_nnt[k] = (float)(1.0 - (double)a.dones[s]);
            s_v[k] = a.values[s];
            s_r[k] = a.extra ? __fadd_rn(a.rewards[s], a.extra[p]) : a.rewards[s];
        }
    }
    __syncthreads();
    const int64_t p = p0 + threadIdx.x;
    if (p >= a.n) return;
    const int k0 = threadIdx.x;
    if (p == a.n - 1) {
        gae_write(a, p, 0.0f, s_v[k0]);
        return;
    }
    const float g = a.gamma, gl = __fmul_rn(a.gamma, a.lambda);
    const int64_t e = (p + a.window < a.n - 2) ? p + a.window : a.n - 2;
    float last = 0.0f;
    for (int k = (int)(e - p0); k >= k0; --k) last = gae_step(last, s_nnt[k + 1], s_v[k + 1], s_r[k + 1], s_v[k], g, gl);
    gae_write(a, p, last, s_v[k0]);
}

// serial fallback: one block walks the array backwards in LDS chunks; lane 0 runs the recurrence
constexpr int SERIAL_CHUNK = 4096;

__global__ void __launch_bounds__(BLOCK) gae_serial_kernel(GaeArgs a) {
    __shared__ float s_nnt[SERIAL_CHUNK + 1], s_v[SERIAL_CHUNK + 1], s_r[SERIAL_CHUNK + 1], s_out[SERIAL_CHUNK];
    __shared__ float carry_s;
    if (threadIdx.x == 0) carry_s = 0.0f;
    const float g = a.gamma, gl = __fmul_rn(a.gamma, a.lambda);
    if (a.n >= 1 && threadIdx.x == 0) gae_write(a, a.n - 1, 0.0f, a.values[src_of(a, a.n - 1)]);
    // positions [lo, hi) computed in this chunk need operands at [lo, hi]
    for (int64_t hi = a.n - 1; hi > 0; hi -= SERIAL_CHUNK) {
        const int64_t lo = hi - SERIAL_CHUNK > 0 ? hi - SERIAL_CHUNK : 0;
        const int cnt = (int)(hi - lo);
        __syncthreads();
        for (int k = threadIdx.x; k <= cnt; k += BLOCK) {
            const int64_t p = lo + k, s = src_of(a, p);
            s_nnt[k] = (float)(1.0 - (double)a.dones[s]);
            s_v[k] = a.values[s];
            s_r[k] = a.extra ? __fadd_rn(a.rewards[s], a.extra[p]) : a.rewards[s];
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            float last = carry_s;
            for (int k = cnt - 1; k >= 0; --k) {
                last = gae_step(last, s_nnt[k + 1], s_v[k + 1], s_r[k + 1], s_v[k], g, gl);
                s_out[k] = last;
            }
            carry_s = last;
        }
        __syncthreads();
        for (int k = threadIdx.x; k < cnt; k += BLOCK) gae_write(a, lo + k, s_out[k], s_v[k]);
    }
}

constexpr int MAX_WINDOW = 8192;  // LDS: 3 x (256 + 8193) floats = 101 KB

// smallest W with (gamma*lambda)^W < 2^-200, or -1 when none fits MAX_WINDOW
int gae_window(float gamma, float lambda) {
    const double c = std::fabs((double)(float)(gamma * lambda));
    if (!(c < 1.0)) return -1;
    if (c == 0.0) return 1;
    const double w = std::ceil(200.0 * std::log(2.0) / -std::log(c));
    return w > MAX_WINDOW ? -1 : (int)(w < 1 ? 1 : w);
}

int launch_gae(GaeArgs a, hipStream_t s) {
    if (a.n <= 0) return 0;
    if (!std::isfinite(a.gamma) || !std::isfinite(a.lambda)) return he_fail_text("he_gae: gamma/lambda not finite");
    a.window = gae_window(a.gamma, a.lambda);
    if (a.window > 0) {
        const size_t lds = 3 * sizeof(float) * (size_t)(BLOCK + a.window + 1);
        const int64_t blocks = (a.n + BLOCK - 1) / BLOCK;
        if (blocks > 0x7fffffff) return he_fail_text("he_gae: too many steps");
        gae_window_kernel<<<(unsigned)blocks, BLOCK, lds, s>>>(a);
    } else {
        gae_serial_kernel<<<1, BLOCK, 0, s>>>(a);
    }
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : he_fail_text(hipGetErrorString(e));
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    char buf[256];
    snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
    return he_fail_text(buf);
}

int check_fields(const he_rollout_field* fields, int num_fields, const char* what) {
    char buf[256];
    if (num_fields < 0 || num_fields > HE_ROLLOUT_MAX_FIELDS || (num_fields > 0 && !fields)) {
        snprintf(buf, sizeof(buf), "%s: num_fields must be in [0, %d]", what, HE_ROLLOUT_MAX_FIELDS);
        return he_fail_text(buf);
    }
    for (int i = 0; i < num_fields; ++i) {
        const he_rollout_field& f = fields[i];
        if (!f.src || !f.dst || f.width <= 0 || (f.src_kind != HE_ROLLOUT_F32 && f.src_kind != HE_ROLLOUT_U8)) {
            snprintf(buf, sizeof(buf), "%s: field %d invalid (null pointer, width <= 0 or unknown kind)", what, i);
            return he_fail_text(buf);
        }
    }
    return 0;
}

}  // namespace

extern "C" int he_rollout_store(const he_rollout_index* ix, const he_rollout_field* fields, int num_fields,
                                int64_t num_rows, const int32_t* env_ids, const uint8_t* mask, int64_t ptr,
                                int32_t step, void* stream) {
    if (!ix || num_rows < 0 || (num_rows > 0 && !env_ids))
        return he_fail_text("he_rollout_store: null index/env_ids or negative rows");
    if (ptr < 0 || ptr > ix->capacity) return he_fail_text("he_rollout_store: ptr outside [0, capacity]");
    if (mask && num_rows > ix->scratch_rows) return he_fail_text("he_rollout_store: more rows than scratch_rows");
    if (int rc = check_fields(fields, num_fields, "he_rollout_store")) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    StoreArgs k{env_ids, mask, num_rows, ptr, ix->capacity, step, ix->num_keys, ix->key_count, ix->key_last,
                ix->row_env, ix->row_rank, ix->scratch, ix->status};
    if (mask) {
        store_keys_masked_kernel<<<1, 1024, 0, s>>>(k);
    } else {
        const int64_t blocks = num_rows > 0 ? (num_rows + BLOCK - 1) / BLOCK : 1;
        store_keys_dense_kernel<<<(unsigned)blocks, BLOCK, 0, s>>>(k);
    }
    if (int rc = check_launch("he_rollout_store")) return rc;
    RowsArgs r{};
    for (int i = 0; i < num_fields; ++i) r.fields.f[i] = fields[i];
    r.rows = num_rows;
    r.ptr = ptr;
    r.capacity = ix->capacity;
    r.scratch = ix->scratch;
    r.mode = mask ? MAP_STORE_MASKED : MAP_STORE_DENSE;
    if (int rc = launch_rows(r, s, num_fields)) return rc;
    return check_launch("he_rollout_store");
}

extern "C" int he_rollout_order(const he_rollout_index* ix, int64_t num_rows, int64_t* idxs, int check_errors,
                                void* stream) {
    if (!ix || num_rows < 0 || num_rows > ix->capacity || (num_rows > 0 && !idxs))
        return he_fail_text("he_rollout_order: null argument or num_rows outside [0, capacity]");
    hipStream_t s = static_cast<hipStream_t>(stream);
    offsets_kernel<<<1, 1024, 0, s>>>(ix->key_count, ix->key_offset, ix->num_keys);
    if (num_rows > 0)
        order_kernel<<<(unsigned)((num_rows + BLOCK - 1) / BLOCK), BLOCK, 0, s>>>(ix->row_env, ix->row_rank,
                                                                                 ix->key_offset, num_rows, idxs);
    if (int rc = check_launch("he_rollout_order")) return rc;
    int32_t bits = 0;
    if (check_errors) {
        hipError_t e = hipMemcpyAsync(&bits, ix->status + 1, sizeof(bits), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return he_fail_text(hipGetErrorString(e));
    }
    // next collection: counters 0, stamps -1, error bits clear
    if (hipMemsetAsync(ix->key_count, 0, sizeof(int32_t) * ix->num_keys, s) != hipSuccess ||
        hipMemsetAsync(ix->key_last, 0xff, sizeof(int32_t) * ix->num_keys, s) != hipSuccess ||
        hipMemsetAsync(ix->status, 0, sizeof(int32_t) * 4, s) != hipSuccess)
        return he_fail_text("he_rollout_order: counter reset failed");
    if (bits & HE_ROLLOUT_ERR_KEY_RANGE) return he_fail_text("he_rollout_order: a stored env id was outside [0, num_keys)");
    if (bits & HE_ROLLOUT_ERR_DUP_KEY) return he_fail_text("he_rollout_order: an env id appeared twice in one store call");
    return 0;
}

extern "C" int he_rollout_gather(const he_rollout_field* fields, int num_fields, const int64_t* idxs,
                                 int64_t num_rows, int32_t num_minibatches, int32_t minibatch_rows,
                                 int32_t bptt_horizon, void* stream) {
    if (num_rows < 0 || (num_rows > 0 && !idxs)) return he_fail_text("he_rollout_gather: null idxs or negative rows");
    if (num_minibatches <= 0 || minibatch_rows <= 0 || bptt_horizon <= 0 ||
        (int64_t)num_minibatches * minibatch_rows * bptt_horizon != num_rows)
        return he_fail_text("he_rollout_gather: num_rows != num_minibatches * minibatch_rows * bptt_horizon");
    if (int rc = check_fields(fields, num_fields, "he_rollout_gather")) return rc;
    RowsArgs r{};
    for (int i = 0; i < num_fields; ++i) r.fields.f[i] = fields[i];
    r.rows = num_rows;
    r.idxs = idxs;
    r.num_mb = num_minibatches;
    r.mb_rows = minibatch_rows;
    r.bptt = bptt_horizon;
    r.mode = MAP_GATHER;
    if (int rc = launch_rows(r, static_cast<hipStream_t>(stream), num_fields)) return rc;
    return check_launch("he_rollout_gather");
}

extern "C" int he_gae(const float* dones, const float* values, const float* rewards, int64_t num_steps, float gamma,
                      float gae_lambda, float* advantages, void* stream) {
    if (num_steps < 0 || (num_steps > 0 && (!dones || !values || !rewards || !advantages)))
        return he_fail_text("he_gae: null argument or negative num_steps");
    GaeArgs a{dones, values, rewards, nullptr, nullptr, num_steps, gamma, gae_lambda, 0, 1, 1, 1, advantages, nullptr};
    return launch_gae(a, static_cast<hipStream_t>(stream));
}

extern "C" int he_gae_minibatch(const float* dones, const float* values, const float* rewards,
                                const float* extra_reward, const int64_t* idxs, int64_t num_steps, float gamma,
                                float gae_lambda, int32_t num_minibatches, int32_t minibatch_rows,
                                int32_t bptt_horizon, float* b_advantages, float* b_returns, void* stream) {
    if (num_steps < 0 || (num_steps > 0 && (!dones || !values || !rewards || !idxs || !b_advantages)))
        return he_fail_text("he_gae_minibatch: null argument or negative num_steps");
    if (num_minibatches <= 0 || minibatch_rows <= 0 || bptt_horizon <= 0 ||
        (int64_t)num_minibatches * minibatch_rows * bptt_horizon != num_steps)
        return he_fail_text("he_gae_minibatch: num_steps != num_minibatches * minibatch_rows * bptt_horizon");
    GaeArgs a{dones, values, rewards, extra_reward, idxs, num_steps, gamma, gae_lambda, 0,
              num_minibatches, minibatch_rows, bptt_horizon, b_advantages, b_returns};
    return launch_gae(a, static_cast<hipStream_t>(stream));
}

// ---------------------------------------------------------------- PHCPufferEnv.step bookkeeping
namespace {
constexpr int EB_THREADS = 256;  // 10 x 256 doubles of LDS for the tree
struct EpisodeArgs {
    int n;
    const float* rew;
    const float* reward_raw;
    const uint8_t* reset;
    const uint8_t* terminate;
    float* rew_out;
    uint8_t* term_out;
    uint8_t* terminals;
    uint8_t* truncations;
    uint8_t* masks;
    float* episode_returns;
    int32_t* episode_lengths;
    float* raw_rewards;
    double* acc;
};
// one workgroup: per-thread strided partial sums, then a fixed-order tree in LDS (deterministic)
__global__ void __launch_bounds__(EB_THREADS) episode_step_kernel(EpisodeArgs a) {
    __shared__ double red[10][EB_THREADS];
    const int tid = threadIdx.x;
    double s[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = tid; i < a.n; i += EB_THREADS) {
        const bool r = a.reset[i] != 0, t = a.terminate[i] != 0;
        const bool term = t && r, trunc = r && !t;
        a.terminals[i] = term;
        a.truncations[i] = trunc;
        a.masks[i] = !trunc;
        const float rw = a.rew[i];
        a.rew_out[i] = rw;
        a.term_out[i] = t;
        const float ret = a.episode_returns[i];
        const int32_t len = a.episode_lengths[i];
        if (r) {
            s[0] += (double)ret;
            s[1] += (double)len;
            s[2] += 1.0;
        }
        s[3] += trunc ? 1.0 : 0.0;
        s[4] += term ? 1.0 : 0.0;
        a.episode_returns[i] = r ? 0.0f : ret + rw;
        a.episode_lengths[i] = r ? 0 : len + 1;
        const float* rr = a.reward_raw + (size_t)i * 5;
#pragma unroll
        for (int k = 0; k < 5; ++k) s[5 + k] += (double)rr[k];
    }
#pragma unroll
    for (int k = 0; k < 10; ++k) red[k][tid] = s[k];
    __syncthreads();
    for (int w = EB_THREADS / 2; w > 0; w >>= 1) {
        if (tid < w)
#pragma unroll
            for (int k = 0; k < 10; ++k) red[k][tid] += red[k][tid + w];
        __syncthreads();
    }
    if (tid < 5) a.acc[tid] += red[tid][0];
    if (tid >= 5 && tid < 10 && a.n > 0) a.raw_rewards[tid - 5] += (float)(red[tid][0] / (double)a.n);
}
}  // namespace

extern "C" int he_episode_step(int32_t num_envs, const float* rew, const float* reward_raw, const uint8_t* reset,
                               const uint8_t* terminate, float* rew_out, uint8_t* term_out, uint8_t* terminals,
                               uint8_t* truncations, uint8_t* masks, float* episode_returns, int32_t* episode_lengths,
                               float* raw_rewards, double* acc, void* stream) {
    if (num_envs < 0) return he_fail_text("he_episode_step: negative num_envs");
    if (num_envs > 0 && (!rew || !reward_raw || !reset || !terminate || !rew_out || !term_out || !terminals ||
                         !truncations || !masks || !episode_returns || !episode_lengths || !raw_rewards || !acc))
        return he_fail_text("he_episode_step: null argument");
    if (num_envs == 0) return 0;
    EpisodeArgs a{num_envs, rew, reward_raw, reset, terminate, rew_out, term_out, terminals, truncations, masks,
                  episode_returns, episode_lengths, raw_rewards, acc};
    episode_step_kernel<<<1, EB_THREADS, 0, static_cast<hipStream_t>(stream)>>>(a);
    return check_launch("he_episode_step");
}
