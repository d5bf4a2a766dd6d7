/*
 * he_oracle_rollout.c -- TEST INFRASTRUCTURE ONLY (see he_oracle.c's header): CPU restatement of
 * the rollout -> trainer handoff, the checker for include/humanoid_rollout.h.
 *
 *   ho_gae          c_gae.pyx:11-32 compute_gae. float32 arithmetic in the Cython module's operation
 *                   order (`1.0 - done` is a C double, rounded to the float `nextnonterminal`);
 *                   compiled with -ffp-contract=off like the reference module's x86-64 build (no FMA).
 *                   PARITY UNPINNED against the reference module (building it here was denied, see
 *                   DESIGN.md §6); checked with closed-form known-answer cases in tests/test_rollout.py.
 *   ho_sort_keys    clean_pufferl/structs.py:128-129: sorted(range(n), key=(env_id, step)), Python's
 *                   stable sort (ties keep store order).
 */
#include <stdint.h>
#include <stdlib.h>

void ho_gae(int64_t n, const float* dones, const float* values, const float* rewards, float gamma, float gae_lambda,
            float* advantages) {
    for (int64_t i = 0; i < n; ++i) advantages[i] = 0.0f;  /* np.zeros */
    float lastgaelam = 0.0f, nextnonterminal, delta;
    for (int64_t t = 0; t < n - 1; ++t) {
        const int64_t t_cur = n - 2 - t, t_next = n - 1 - t;
        nextnonterminal = (float)(1.0 - (double)dones[t_next]);
        delta = rewards[t_next] + gamma * values[t_next] * nextnonterminal - values[t_cur];
        lastgaelam = delta + gamma * gae_lambda * nextnonterminal * lastgaelam;
        advantages[t_cur] = lastgaelam;
    }
}

typedef struct { int64_t env, step, idx; } key_t3;

static int cmp_key(const void* a, const void* b) {
    const key_t3* x = (const key_t3*)a;
    const key_t3* y = (const key_t3*)b;
    if (x->env != y->env) return x->env < y->env ? -1 : 1;
    if (x->step != y->step) return x->step < y->step ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);  /* stability: store order breaks ties */
}

void ho_sort_keys(int64_t n, const int64_t* env_id, const int64_t* step, int64_t* idxs) {
    key_t3* k = (key_t3*)malloc(sizeof(key_t3) * (size_t)(n > 0 ? n : 1));
    for (int64_t i = 0; i < n; ++i) { k[i].env = env_id[i]; k[i].step = step[i]; k[i].idx = i; }
    qsort(k, (size_t)n, sizeof(key_t3), cmp_key);
    for (int64_t i = 0; i < n; ++i) idxs[i] = k[i].idx;
    free(k);
}
