#!/bin/bash
# Build an A/B variant of libsd_hip_cas.so: copy csrc to a scratch dir, apply a patch (argument
# 2: a python script, or a shell command run in the copy's csrc, e.g.
# "python3 $R/tools/patch_define.py SD_K2_BLOCK_KEY 0"), build, and place the library at
# tools/ablib/<name>.so.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
PATCH=$2
W=$(mktemp -d /tmp/sdvar.XXXXXX)
mkdir -p "$W/pkg" "$W/include"
cp -r "$R/spacedrive_amd/csrc" "$W/pkg/csrc"
cp "$R/include/sd_hip_cas.h" "$W/include/"
rm -rf "$W/pkg/csrc/build"
if [ -f "$PATCH" ]; then (cd "$W/pkg/csrc" && python3 "$PATCH"); else (cd "$W/pkg/csrc" && R="$R" bash -c "$PATCH"); fi
make -s -C "$W/pkg/csrc" -j8 OUT="$W/lib.so" >/dev/null
mkdir -p "$R/tools/ablib"
cp "$W/lib.so" "$R/tools/ablib/$NAME.so"
rm -rf "$W"
echo "built tools/ablib/$NAME.so"
