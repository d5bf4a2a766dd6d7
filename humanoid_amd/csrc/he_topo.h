// he_topo.h -- static articulation tables derived once from the model on the host and read by
// the physics kernel (wave-uniform reads go through the scalar cache).
#pragma once
#include <stdint.h>

#include "../../include/humanoid_engine.h"

#define HE_MAX_CHAIN 30    // longest root->dof chain: 6 root dofs + 8 bodies x 3
#define HE_NNZ_MAX 1280    // packed lower-triangular sparse mass matrix (1221 for SMPL)
#define HE_MAX_TRI 435     // pairs (i,j), j<=i<29 of one elimination step
#define HE_MAX_BOXES 5     // box geoms: one 8-lane corner group each in lanes 24..63 (SMPL: 4)

struct PhysTopo {
    int32_t nnz;
    int32_t num_levels;              // dof levels by chain length (1..30)
    int8_t dof_parent[HE_NUM_GEN];
    int8_t dof_body[HE_NUM_GEN];
    int8_t dof_nanc[HE_NUM_GEN];     // chain length incl. self
    int16_t row_start[HE_NUM_GEN];   // H(i, j) at row_start[i] + position of j in chain(i)
    int8_t dof_chain[HE_NUM_GEN][HE_MAX_CHAIN];
    int8_t body_dof0[HE_NUM_BODIES];
    int8_t body_depth[HE_NUM_BODIES];
    int8_t body_chain[HE_NUM_BODIES][9];  // root-first body chain incl. self
    uint32_t anc_mask[HE_NUM_BODIES];     // bit a: a is ancestor-or-self of b
    uint32_t sub_mask[HE_NUM_BODIES];     // bit d: d in subtree(b)
    int16_t level_start[HE_MAX_CHAIN + 1];
    int8_t level_dofs[HE_NUM_GEN];        // dofs grouped by chain length
    uint8_t tri_i[HE_MAX_TRI], tri_j[HE_MAX_TRI];
    uint8_t ent_row[HE_NNZ_MAX];          // packed entry -> row of the sparse mass matrix
    int8_t body_last_dof[HE_NUM_BODIES];  // chain(body_last_dof[b]) = all dofs on b's chain
    int32_t num_boxes;
    int8_t corner_body[64];  // lane 24 + 8k + c: corner c of the k-th box geom's body (-1: none)
};

#ifdef __cplusplus
static inline void he_build_topo(const he_model& m, PhysTopo& t) {
    for (int i = 0; i < 6; ++i) { t.dof_parent[i] = (int8_t)(i - 1); t.dof_body[i] = 0; }
    t.body_dof0[0] = 0;
    for (int b = 1; b < HE_NUM_BODIES; ++b) {
        int d0 = 6 + 3 * (b - 1);
        t.body_dof0[b] = (int8_t)d0;
        int p = m.parents[b];
        int plast = p == 0 ? 5 : 6 + 3 * (p - 1) + 2;
        for (int c = 0; c < 3; ++c) {
            t.dof_parent[d0 + c] = (int8_t)(c == 0 ? plast : d0 + c - 1);
            t.dof_body[d0 + c] = (int8_t)b;
        }
    }
    int off = 0;
    for (int i = 0; i < HE_NUM_GEN; ++i) {
        int chain[HE_MAX_CHAIN + 8], n = 0;
        for (int j = i; j >= 0; j = t.dof_parent[j]) chain[n++] = j;
        t.dof_nanc[i] = (int8_t)n;
        for (int k = 0; k < HE_MAX_CHAIN; ++k) t.dof_chain[i][k] = (int8_t)(k < n ? chain[n - 1 - k] : -1);
        t.row_start[i] = (int16_t)off;
        off += n;
    }
    t.nnz = off;
    for (int b = 0; b < HE_NUM_BODIES; ++b) {
        int chain[16], n = 0;
        for (int a = b; a >= 0; a = (a == 0 ? -1 : m.parents[a])) chain[n++] = a;
        t.body_depth[b] = (int8_t)(n - 1);
        for (int k = 0; k < 9; ++k) t.body_chain[b][k] = (int8_t)(k < n ? chain[n - 1 - k] : -1);
        uint32_t am = 0;
        for (int k = 0; k < n; ++k) am |= 1u << chain[k];
        t.anc_mask[b] = am;
    }
    for (int b = 0; b < HE_NUM_BODIES; ++b) {
        uint32_t sm = 0;
        for (int d = 0; d < HE_NUM_BODIES; ++d)
            if (t.anc_mask[d] >> b & 1u) sm |= 1u << d;
        t.sub_mask[b] = sm;
    }
    int cnt = 0, lvl = 0;
    for (int len = 1; len <= HE_MAX_CHAIN; ++len) {
        t.level_start[len - 1] = (int16_t)cnt;
        for (int i = 0; i < HE_NUM_GEN; ++i)
            if (t.dof_nanc[i] == len) t.level_dofs[cnt++] = (int8_t)i;
        if (cnt > t.level_start[len - 1]) lvl = len;
    }
    t.level_start[HE_MAX_CHAIN] = (int16_t)cnt;
    t.num_levels = lvl;
    for (int i = 0; i < HE_NUM_GEN; ++i)
        for (int k = 0; k < t.dof_nanc[i]; ++k) t.ent_row[t.row_start[i] + k] = (uint8_t)i;
    for (int b = 0; b < HE_NUM_BODIES; ++b) t.body_last_dof[b] = (int8_t)(b == 0 ? 5 : 6 + 3 * (b - 1) + 2);
    int p = 0;
    for (int i = 0; i < 29 && p < HE_MAX_TRI; ++i)
        for (int j = 0; j <= i && p < HE_MAX_TRI; ++j) { t.tri_i[p] = (uint8_t)i; t.tri_j[p] = (uint8_t)j; ++p; }
    t.num_boxes = 0;
    for (int l = 0; l < 64; ++l) t.corner_body[l] = -1;
    for (int b = 0; b < HE_NUM_BODIES; ++b)
        if (m.geom_type[b] == HE_GEOM_BOX) {
            if (t.num_boxes < HE_MAX_BOXES)
                for (int c = 0; c < 8; ++c) t.corner_body[HE_NUM_BODIES + 8 * t.num_boxes + c] = (int8_t)b;
            ++t.num_boxes;
        }
}
#endif

static_assert(sizeof(PhysTopo) % 4 == 0, "PhysTopo is copied to LDS in 4-byte words");
