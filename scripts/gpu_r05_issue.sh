#!/bin/bash
# Round 5: host time of a bench step's parts (tools/probe_issue.py)
OUT=${OUT:-r05i}
exec scripts/gpu_run.sh $OUT \
  issue 300 python3 tools/probe_issue.py
