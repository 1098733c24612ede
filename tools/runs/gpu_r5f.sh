#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" && mkdir -p gpurun_out/r5
bash tools/runs/gpu_r5e.sh || exit $?
bash tools/runs/gpu_r5d.sh
