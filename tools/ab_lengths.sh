#!/bin/bash
# Interleaved bench.py A/B: base-6 record lengths (default for input6) vs 3-bit fields (--lengths bits3).
REPS=${REPS:-3} STEPS=${STEPS:-300} AB_ENV=X=1 AB_ARGS="--lengths bits3" exec bash tools/ab_env.sh
