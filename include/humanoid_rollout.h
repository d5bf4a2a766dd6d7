/*
 * humanoid_rollout.h -- C ABI of the rollout -> trainer handoff on the device,
 * exported by the same libhumanoid_engine.so (gfx950).
 *
 * It replaces the host round trips between PHCPufferEnv.step and the PPO update in puffer-phc
 * (paths under packages/puffer-phc/puffer_phc/):
 *   - Experience.store            clean_pufferl/structs.py:108-126  (6 D2H copies per step)
 *   - Experience.sort_training_data clean_pufferl/structs.py:128-142  (Python `sorted` of (env, step))
 *   - Experience.flatten_batch      clean_pufferl/structs.py:144-160  (host gathers + H2D)
 *   - compute_gae                   c_gae.pyx:11-32 (Cython, host), called at clean_pufferl/core.py:245-247
 *   - the advantage/return layout   clean_pufferl/core.py:249-256
 *
 * Conventions as humanoid_engine.h: 0 = success, he_last_error() for the text; every data pointer
 * is a DEVICE pointer (the he_rollout_index / he_rollout_field structs themselves are host memory);
 * `stream` is a hipStream_t; nothing synchronises the host.
 */
#ifndef HUMANOID_ROLLOUT_H
#define HUMANOID_ROLLOUT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HE_ROLLOUT_MAX_FIELDS 8
#define HE_ROLLOUT_F32 0         /* source rows are float32 */
#define HE_ROLLOUT_U8 1          /* source rows are uint8/bool, stored as 0.0f / 1.0f */

/* status[1] error bits, set by he_rollout_store and reported (then cleared) by he_rollout_order */
#define HE_ROLLOUT_ERR_KEY_RANGE 1   /* an env id outside [0, num_keys) */
#define HE_ROLLOUT_ERR_DUP_KEY 2     /* the same env id twice in one store call */

/* One stored column group: `width` values per row. In he_rollout_store `src` is the per-step
 * tensor [num_rows, width] and `dst` the flat buffer [capacity, width]; in he_rollout_gather `src`
 * is the flat buffer and `dst` the minibatch-ordered buffer [capacity, width]. */
typedef struct he_rollout_field {
    const void* src;
    float* dst;
    int32_t width;
    int32_t src_kind;            /* HE_ROLLOUT_F32 or HE_ROLLOUT_U8 */
} he_rollout_field;

/* Device bookkeeping that stands in for Experience.sort_keys (structs.py:121): every stored row
 * keeps its env id and its rank among that env's rows, so the (env_id, step) order is a counting
 * sort. All arrays are caller-owned device memory; key_count = 0 and key_last = -1 initially. */
typedef struct he_rollout_index {
    int32_t num_keys;            /* env ids lie in [0, num_keys) */
    int32_t reserved;
    int64_t capacity;            /* Experience.batch_size */
    int64_t scratch_rows;        /* >= rows per store call */
    int32_t* key_count;          /* [num_keys] rows stored per env so far */
    int32_t* key_last;           /* [num_keys] step of the env's last store (-1: none) */
    int32_t* key_offset;         /* [num_keys] scratch of he_rollout_order */
    int32_t* row_env;            /* [capacity] env id of each stored row */
    int32_t* row_rank;           /* [capacity] rank of the row among its env's rows */
    int32_t* scratch;            /* [scratch_rows] destination row of each source row */
    int32_t* status;             /* [4]: rows stored by the last call, error bits, 0, 0 */
} he_rollout_index;

/* Experience.store (structs.py:108-126): rows i with mask[i] != 0 (mask NULL = all rows), in
 * order, go to flat rows ptr, ptr+1, ... up to capacity (the `indices[: batch_size - ptr]` cut);
 * status[0] receives how many were stored. `step` is Experience.step (one per call). */
int he_rollout_store(const he_rollout_index* ix, const he_rollout_field* fields, int num_fields,
                     int64_t num_rows, const int32_t* env_ids, const uint8_t* mask, int64_t ptr,
                     int32_t step, void* stream);

/* Experience.sort_training_data (structs.py:128-131): idxs[0:num_rows] = the stored rows sorted by
 * (env_id, step), the order Python's stable `sorted` gives; then clears the per-env counters for
 * the next collection. The store error bits are checked here, once per batch: with check_errors
 * non-zero this call waits for the stream and fails if a store reported HE_ROLLOUT_ERR_*
 * (the reference syncs at the same point, structs.py:131-136); rows with a bad env id are never
 * written out of bounds either way. */
int he_rollout_order(const he_rollout_index* ix, int64_t num_rows, int64_t* idxs, int check_errors, void* stream);

/* Experience.flatten_batch (structs.py:144-160): for every field, dst row d = src row idxs[p]
 * where d enumerates [num_minibatches][minibatch_rows][bptt_horizon] and p is the same element in
 * the sorted order [minibatch_rows][num_minibatches][bptt_horizon] (the b_idxs transpose,
 * structs.py:130-137). num_rows = num_minibatches * minibatch_rows * bptt_horizon. */
int he_rollout_gather(const he_rollout_field* fields, int num_fields, const int64_t* idxs, int64_t num_rows,
                      int32_t num_minibatches, int32_t minibatch_rows, int32_t bptt_horizon, void* stream);

/* compute_gae (c_gae.pyx:11-32) over flat float32 arrays of num_steps: advantages[num_steps-1] = 0,
 * and the reverse recurrence in float32 with the Cython module's operation order. */
int he_gae(const float* dones, const float* values, const float* rewards, int64_t num_steps, float gamma,
           float gae_lambda, float* advantages, void* stream);

/* core.py:213-256 fused: GAE over the sorted rows (dones/values/rewards are the flat storage-order
 * buffers, gathered through idxs; extra_reward, may be NULL, is added per sorted position as
 * `rewards_np + adversarial_reward_np` is), written straight into the minibatch layout:
 * b_advantages[d] = adv[p], b_returns[d] = adv[p] + values[idxs[p]] (d, p as he_rollout_gather). */
int he_gae_minibatch(const float* dones, const float* values, const float* rewards, const float* extra_reward,
                     const int64_t* idxs, int64_t num_steps, float gamma, float gae_lambda, int32_t num_minibatches,
                     int32_t minibatch_rows, int32_t bptt_horizon, float* b_advantages, float* b_returns,
                     void* stream);

/* PHCPufferEnv.step episode bookkeeping in one launch (clean_pufferl/env.py:120-160, replacing its
 * nonzero / tolist / isin host round trips and the per-step torch ops of the device mirror). For
 * env i with r = reset[i], t = terminate[i] (0/1 bytes): terminals[i] = t & r, truncations[i] =
 * r & !t, masks[i] = !truncations[i]; rew_out[i] = rew[i] and term_out[i] = t (the step's returned
 * copies, env.py:121); acc[0..4] += the sums over reset envs of episode_returns, episode_lengths,
 * 1, truncation, termination (double, env.py:137-148's info lists reduced on the device); then
 * episode_returns[i] = r ? 0 : episode_returns[i] + rew[i], episode_lengths[i] = r ? 0 :
 * episode_lengths[i] + 1 (env.py:140-141, 159-160), and raw_rewards[k] += mean_i reward_raw[i][k]
 * for k < 5 (env.py:124). One workgroup, fixed-order sums: the result is deterministic. Device
 * pointers; num_envs >= 0. */
int he_episode_step(int32_t num_envs, const float* rew, const float* reward_raw, const uint8_t* reset,
                    const uint8_t* terminate, float* rew_out, uint8_t* term_out, uint8_t* terminals,
                    uint8_t* truncations, uint8_t* masks, float* episode_returns, int32_t* episode_lengths,
                    float* raw_rewards, double* acc, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* HUMANOID_ROLLOUT_H */
