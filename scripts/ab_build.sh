#!/bin/bash
# Build a variant of libspe.so for kernel A/B timing: ablate/<name>/libspe.so with extra hipcc
# flags (e.g. -DSPE_ATTN_OCC=2).  Load it with SPE_LIB_PATH=ablate/<name>/libspe.so.
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/ablate/$NAME"
make -s -j8 -C "$ROOT/satellite-pose-estimation_amd/csrc" OBJDIR="$ROOT/ablate/$NAME/obj" OUT="$ROOT/ablate/$NAME/libspe.so" EXTRA="$*"
