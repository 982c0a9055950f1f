#!/bin/bash
# Build a variant of the product library for an A/B session (CPU side, before gpurun):
#   bash scripts/build_variant.sh <name> [git-rev | -] [EXTRA compiler flags...]
# <git-rev>: build the csrc/ sources of that revision (e.g. HEAD for the committed baseline); "-": the working tree.
# Output: build_ab/libgsr_hip_<name>.so (git-ignored, travels to the box with the snapshot).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
REV=${2:--}
shift 2 || shift $#
mkdir -p "$ROOT/build_ab"
SRC="$ROOT/threestudio-3dgs_amd/csrc"
if [ "$REV" != "-" ]; then
  TMP=$(mktemp -d)
  git -C "$ROOT" archive "$REV" threestudio-3dgs_amd/csrc include | tar -x -C "$TMP"
  SRC="$TMP/threestudio-3dgs_amd/csrc"
fi
make -s -j 8 -C "$SRC" OBJDIR="$ROOT/build_ab/obj_$NAME" OUT="$ROOT/build_ab/libgsr_hip_$NAME.so" EXTRA="$*"
echo "built build_ab/libgsr_hip_$NAME.so"
