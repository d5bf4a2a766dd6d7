#!/bin/bash
# Round-4 A/B set: four-lane readlane blocks for the dot-product broadcasts (HE_RL4) and the L^-T
# pipeline's group size (HE_LT_GROUP 6 / 8 / 12): interleaved phase profiles of the stamp variants,
# then bit-identity and 4 interleaved bench passes of the product variants. Stops at the first failure.
set -o pipefail
bash tools/gpu_r04_p.sh phbase phrl4 phlt8 &&
SKIP_TESTS=1 AB_PASSES="1 2 3 4" bash tools/gpu_ab_ident.sh humanoid_amd/_variants/rl4.so humanoid_amd/_variants/lt8.so humanoid_amd/_variants/lt6.so humanoid_amd/_variants/lt12.so
