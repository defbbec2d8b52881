#!/bin/bash
# --memory_first: SwiGLU output kept per layer (DLT_S_REFILL=0) vs rewritten by the backward.
set -u
VARIANTS="base:X=0 keep_s:DLT_S_REFILL=0" REPS=${REPS:-3} BENCH_ARGS="--memory_first" bash tools/ab/env_ab.sh
