#!/bin/bash
# An A/B build of the library with compile-time overrides of the tuning constants
# (the product library has no runtime switches):
#   [ONLY="k_bitonic k_fold"] scripts/ab_build.sh NAME -DFLTEE_SORT_LATEPF_KEY=1 ...
# -> fl-tee_amd/lib/ab/libfltee_agg_NAME.so, loaded by a run with FLTEE_LIB=<that path>
#    (scripts/ab_env.py c5 FLTEE_LIB=fl-tee_amd/lib/ab/libfltee_agg_NAME.so)
# ONLY: the sources the overrides touch; the other objects are copied from the product
# build (fl-tee_amd/build) instead of being recompiled.
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name="$1"; shift
B="$ROOT/fl-tee_amd/build_ab/$name"
mkdir -p "$B"
if [ -n "${ONLY:-}" ]; then
  for o in "$ROOT"/fl-tee_amd/build/*.o; do
    base=$(basename "$o" .o)
    case " $ONLY version " in *" $base "*) continue ;; esac
    cp -p "$o" "$B/"
  done
fi
make -C "$ROOT/fl-tee_amd" -j8 BUILD="$B" LIB="$ROOT/fl-tee_amd/lib/ab/libfltee_agg_$name.so" TUNE="$*"
