#!/bin/bash
# round 6: the backward's LDS cap 12 KiB (default) against 8 KiB, and with the Localizer lane's
# streaming loads (nt=1), driver command, same box, interleaved; the bench with its live-V
# counters restarted after the step window (the roofline's bytes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
SWEEP="base;bwd_lds=8192;bwd_lds=8192,nt=1;base;bwd_lds=8192" BENCH_ARGS="--steps 20 --warmup 5" bash tools/ctx_sweep.sh
