#!/bin/bash
# Builds libvvcr from a git revision (default HEAD) into vvc_amd/libvvcr_old.so for A/B runs
# (tools/mc_run.sh picks it up when present). Uses a temporary worktree; the working tree is untouched.
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/vvcr_ab.XXXX)
git -C "$ROOT" worktree add -q --detach "$WT" "$REV"
(cd "$WT" && python -c "from vvc_amd import build as B; B.build_lib()")
cp "$WT/vvc_amd/libvvcr.so" "$ROOT/vvc_amd/libvvcr_old.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built $REV -> vvc_amd/libvvcr_old.so"
