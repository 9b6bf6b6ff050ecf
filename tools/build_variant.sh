#!/bin/bash
# Build an A/B variant of libkdpt.so into ab/NAME.so with extra compile flags (e.g. -DKDPT_TRACE_BLOCK=512);
# the host objects come from the regular in-tree build (run _build first).
#   bash tools/build_variant.sh NAME [hipcc flags...]
# KDPT_REV=<git rev>: build that revision's kernels instead of the working tree's (its csrc/ is exported to
# build/ab/src-<rev>), e.g. the base of an A/B against uncommitted changes.
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/ab" "$ROOT/build/ab"
SRC="$ROOT/kdtreepathtraceroptimization_amd/csrc"
if [ -n "$KDPT_REV" ]; then
  SRC="$ROOT/build/ab/src-$KDPT_REV"
  rm -rf "$SRC" && mkdir -p "$SRC"
  git -C "$ROOT" archive "$KDPT_REV" kdtreepathtraceroptimization_amd/csrc include | tar -x -C "$SRC"
  SRC="$SRC/kdtreepathtraceroptimization_amd/csrc"
fi
# the product's device code-generation flags (scheduler), so a variant differs from libkdpt.so only by "$@"
# (KDPT_DEVICE_FLAGS overrides them, e.g. KDPT_DEVICE_FLAGS=" " for the default machine scheduler)
DEVICE_FLAGS=${KDPT_DEVICE_FLAGS:-$(cd "$ROOT" && python3 -m kdtreepathtraceroptimization_amd._build --device-flags)}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -I "$ROOT/include" $DEVICE_FLAGS "$@" \
  -c "$SRC/kdpt_runtime.hip" -o "$ROOT/build/ab/$NAME.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/ab/$NAME.so" "$ROOT/build/ab/$NAME.o" \
  "$ROOT/build/kd_build.o" "$ROOT/build/scene_host.o" "$ROOT/build/image_io.o"
echo "ab/$NAME.so"
