#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for the hot path's access shapes (tools/membench/pmccal):
# one --pmc pass per counter, never combined with tracing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 60 tools/membench/pmccal > gpurun_out/pmccal.log 2>&1 || exit $?
cat gpurun_out/pmccal.log
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmccal_fetch -o pmc --output-format csv -- tools/membench/pmccal > /dev/null 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmccal_write -o pmc --output-format csv -- tools/membench/pmccal > /dev/null 2>&1 || exit $?
echo done
