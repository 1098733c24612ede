#!/bin/bash
# profiles/<TAG>/ from the gpurun_out/ of `tools/profile.sh TAG` (run on the GPU box): kernel
# trace summaries of the four bench runs and the PMC JSON files bench.py reads (PMC_ROUND).
# The sharded traces end with the bench's secondary schedules (short bulk-synchronous runs of
# the other exchange designs): their step markers are skipped.
set -e
TAG=${1:?tag}
cd "$(dirname "$0")/.."
O=gpurun_out
P=profiles/$TAG
mkdir -p $P
F=$O/pmc_${TAG}_fetch/pmc_counter_collection.csv
W=$O/pmc_${TAG}_write/pmc_counter_collection.csv
# the fused bench runs its 20 timed steps, then the step-window replay of the same 20 batches
# (round 6), an untimed diagnostic pass over them and 20 host-idle calls (bench.py): the window
# is the timed steps, 60 markers back —
# the 19 intervals between the 20 timed steps' markers (a 20th would reach back over the
# host's sync between the warm-up and the timed loop)
DFX_STEP_SKIP=60 python3 tools/prof_summary.py $O/prof_${TAG}_fused/trace_kernel_trace.csv 19 \
  $F $W > $P/kernel_summary_pipelined.md
DFX_STEP_SKIP=60 python3 tools/prof_summary.py $O/prof_${TAG}_serial/trace_kernel_trace.csv 19 \
  $F $W > $P/kernel_summary_serial.md
DFX_STEP_MARKER=k_split_worker_finalize DFX_STEP_SKIP=44 python3 tools/prof_summary.py \
  $O/prof_${TAG}_split/trace_kernel_trace.csv 20 $O/pmc_${TAG}_fetch_split/pmc_counter_collection.csv \
  $O/pmc_${TAG}_write_split/pmc_counter_collection.csv > $P/kernel_summary_split_pipelined.md
DFX_STEP_MARKER=k_dist_worker_finalize DFX_STEP_SKIP=44 python3 tools/prof_summary.py \
  $O/prof_${TAG}_a2a/trace_kernel_trace.csv 20 > $P/kernel_summary_a2a_pipelined.md
python3 tools/pmc_json.py $F $W $P/pmc_hbm.json 3 $TAG
python3 tools/pmc_json.py $O/pmc_${TAG}_fetch_split/pmc_counter_collection.csv \
  $O/pmc_${TAG}_write_split/pmc_counter_collection.csv $P/pmc_hbm_split.json 3 $TAG
U=$(grep -o '"mean_unique_keys": [0-9.]*' $O/pmc_${TAG}_req.log | head -1 | awk '{print $2}')
python3 tools/pmc_requests.py $O/pmc_${TAG}_req/pmc_counter_collection.csv "$U" 3900000 \
  $P/pmc_requests.json $TAG
ls $P
# the other configs (tools/profile_configs.sh TAG), when their runs are here: the same window
# (19 intervals between the 20 timed steps' markers, 60 markers back)
for c in c2 c5 c4shard; do
  [ -f $O/prof_${TAG}_$c/trace_kernel_trace.csv ] || continue
  CF=$O/pmc_${TAG}_${c}_FETCH_SIZE/pmc_counter_collection.csv
  CW=$O/pmc_${TAG}_${c}_WRITE_SIZE/pmc_counter_collection.csv
  DFX_STEP_SKIP=60 python3 tools/prof_summary.py $O/prof_${TAG}_$c/trace_kernel_trace.csv 19 \
    $CF $CW > $P/kernel_summary_$c.md
  python3 tools/pmc_json.py $CF $CW $P/pmc_hbm_$c.json 3 $TAG
done
ls $P
