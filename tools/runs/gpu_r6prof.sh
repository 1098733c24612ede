#!/bin/bash
# round 6 profiles of the tree at 309227b: kernel traces of the bench (fused, Localizer lane
# serialised, split, a2a) and the separate PMC passes (tools/profile.sh r6), then the other
# configs' traces + PMC (tools/profile_configs.sh r6); tools/prof_collect.sh r6 summarises them
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
bash tools/profile.sh r6 || exit $?
bash tools/profile_configs.sh r6 || exit $?
