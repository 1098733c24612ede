#!/bin/bash
# round-5 closing traces and PMC passes on the final kernels: C3 (fused, serial, split, a2a)
# and the other configs (c2, c5, c4shard); tools/prof_collect.sh r5 turns them into profiles/r5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/profile.sh r5 && CONFIGS="c2 c5 c4shard" bash tools/profile_configs.sh r5
