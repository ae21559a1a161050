#!/bin/bash
# Build the C-ABI library as it was at a commit (or with extra defines) into build/rtw_<name>.so, for same-box A/Bs
# against the in-tree library (tools/ab_c2.sh ... build/rtw_<name>.so).  Runs here (hipcc cross-compiles gfx950);
# prints the build's rtw_build_id so a profiles/ README can name both sides.
#   tools/build_at.sh <commit> <name> ["-DRTW_WALK_PREFETCH ..."]
set -eu
COMMIT=$1; NAME=$2; DEFS=${3:-}
REPO=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/rtw_wt_XXXX)
git -C "$REPO" worktree add --detach "$WT" "$COMMIT" > /dev/null
trap 'git -C "$REPO" worktree remove --force "$WT"' EXIT
mkdir -p "$REPO/build"
make -C "$WT/zig-raytracing-weekend_amd/csrc" -j8 OBJDIR=obj_at OUT="$REPO/build/rtw_$NAME.so" EXTRA_DEFS="$DEFS" > /dev/null
python3 - "$REPO/build/rtw_$NAME.so" "$COMMIT" "$DEFS" <<'PY'
import ctypes, sys
L = ctypes.CDLL(sys.argv[1])
bid = L.rtw_build_id() if hasattr(L, "rtw_build_id") else None
if bid is not None:
    L.rtw_build_id.restype = ctypes.c_char_p
    bid = L.rtw_build_id().decode()
print(f"{sys.argv[1]}: commit {sys.argv[2]} defs '{sys.argv[3]}' build_id {bid}")
PY
