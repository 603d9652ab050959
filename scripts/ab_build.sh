#!/bin/bash
# An A/B build of the library with compile-time overrides of the tuning constants
# (the product library has no runtime switches):
#   scripts/ab_build.sh NAME -DFLTEE_SORT_LATEPF_KEY=1 ...
# -> fl-tee_amd/lib/ab/libfltee_agg_NAME.so, loaded by a run with FLTEE_LIB=<that path>
#    (scripts/ab_env.py c5 FLTEE_LIB=fl-tee_amd/lib/ab/libfltee_agg_NAME.so)
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name="$1"; shift
make -C "$ROOT/fl-tee_amd" -j8 BUILD="$ROOT/fl-tee_amd/build_ab/$name" \
     LIB="$ROOT/fl-tee_amd/lib/ab/libfltee_agg_$name.so" TUNE="$*"
