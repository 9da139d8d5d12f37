#!/bin/bash
# Round-5 final-tree evidence set: GPU tests, smoke, bench, the bench under
# rocprofv3 --kernel-trace --stats (tools/gpu_check.sh), PMC traffic of the
# FEC kernels (FETCH_SIZE / WRITE_SIZE, one counter per pass), the protection
# kernels' instruction counts and their stall picture.  Steps chained with
# &&: the first failure ends the call.
# Usage: tools/gpu_r5final.sh <tag>
TAG=${1:-r5f}
bash tools/gpu_check.sh "$TAG" &&
bash tools/pmc.sh "$TAG" &&
bash tools/pmc_protect.sh "$TAG" &&
bash tools/pmc_aead_stall.sh "$TAG"
