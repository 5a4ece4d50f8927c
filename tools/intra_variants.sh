#!/bin/bash
# Builds libvvcr variants for k_intra A/B runs: vvc_amd/libvvcr_v<name>.so from the working tree with extra
# defines. Usage: tools/intra_variants.sh name1 "-DA=1 -DB" name2 "-DC" ...   (run here, not on the box)
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  python - "$ROOT" "$name" "$defs" <<'PY'
import sys, os
root, name, defs = sys.argv[1], sys.argv[2], sys.argv[3]
sys.path.insert(0, root)
from vvc_amd import build as B
B.build_lib(extra=defs.split(), obj_dir=os.path.join(root, "build", "var_" + name), lib=os.path.join(root, "vvc_amd", "libvvcr_v%s.so" % name))
print("built", name, defs)
PY
done
