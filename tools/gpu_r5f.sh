#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/r5
bash tools/gpu_r5e.sh || exit $?
bash tools/gpu_r5d.sh
