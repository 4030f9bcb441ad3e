#!/bin/bash
# development (round 2): K2 ring-2 occupancy probe
scripts/gpu_run.sh r02al q1 120 tools/micro_k2 q :: q2 120 tools/micro_k2 q
