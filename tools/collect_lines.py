#!/usr/bin/env python3
"""append bench.py lines from gpurun_out logs to profiles/<round>/bench_lines.jsonl:
collect_lines.py ROUND NOTE LOG... (each log's last JSON line, with its file name and the note)"""
import json
import os
import sys

rnd, note, logs = sys.argv[1], sys.argv[2], sys.argv[3:]
out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", rnd,
                   "bench_lines.jsonl")
with open(out, "a") as f:
    for lg in logs:
        try:
            line = json.loads(open(lg).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        f.write(json.dumps({"file": os.path.relpath(lg, "gpurun_out"), "note": note,
                            "line": line}) + "\n")
print(out)
