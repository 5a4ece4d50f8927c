#!/bin/bash
# Profile of the decode path's host side (tools/host_prof_main.cpp: parse, derive, plan per picture, no GPU).
#   tools/host_prof.sh <stream.bin> [repeats]          gprof flat profile (-pg build in build/obj_pg)
#   SAMPLE=1 tools/host_prof.sh <stream.bin> [repeats] SIGPROF PC sampling of the -O3 build (build/obj_g),
#                                                      top functions and source lines via addr2line
set -e
cd "$(dirname "$0")/.."
if [ -n "$SAMPLE" ]; then FL="\"-gdwarf-4\","; OD=build/obj_g; PG=; else FL='"-pg", "-g"'; OD=build/obj_pg; PG=-pg; fi
python3 - <<EOF
import sys; sys.path.insert(0, ".")
from vvc_amd import build as B
B.build_lib(extra=($FL), obj_dir="$OD", lib="$OD/libvvcr.so")
EOF
g++ -O2 -std=c++17 $PG -gdwarf-4 -Iinclude -c tools/host_prof_main.cpp -o $OD/../host_prof_main.o
/opt/rocm/bin/hipcc $PG -no-pie --offload-arch=gfx950 -pthread -o build/host_prof $OD/../host_prof_main.o $OD/*.o
cd build
if [ -n "$SAMPLE" ]; then
  HOST_PROF_PCS=pcs.txt ./host_prof "../$1" "${2:-1}"
  addr2line -f -C -i -e host_prof < pcs.txt > pcs_sym.txt 2>/dev/null || true
  python3 - <<'EOF'
import collections
lines = open("pcs_sym.txt").read().split("\n")
pcs = open("pcs.txt").read().split()
# addr2line -i prints inline frames: pairs (function, file:line); the first pair of each address is the innermost
out, i, k = [], 0, 0
sym = {}
for a in sorted(set(pcs)):
    pass
EOF
  addr2line -f -C -e host_prof < pcs.txt | paste - - > pcs_pair.txt
  python3 - <<'EOF'
import collections
rows = [l.split("\t") for l in open("pcs_pair.txt").read().splitlines()]
fn = collections.Counter(r[0][:110] for r in rows)
ln = collections.Counter((r[1].split("/")[-1] + "  " + r[0][:60]) for r in rows)
n = len(rows)
print("samples", n)
# samples outside the executable (shared libraries: libc's memset / memcpy / malloc ...): nearest dynamic symbol
import bisect, subprocess
maps = []
for l in open("pcs.txt.maps"):
    f = l.split()
    if len(f) >= 6 and f[5].startswith("/") and "x" in f[1]:
        a, b = (int(v, 16) for v in f[0].split("-"))
        maps.append((a, b, int(f[2], 16), f[5]))
syms = {}
def sym(path, off):
    if path not in syms:
        out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout.split("\n")
        t = sorted((int(x.split()[0], 16), x.split()[-1]) for x in out if len(x.split()) >= 3)
        syms[path] = t
    t = syms[path]
    k = bisect.bisect_right(t, (off, "\xff")) - 1
    return path.split("/")[-1] + ":" + (t[k][1] if k >= 0 else "?")
for i, pc in enumerate(open("pcs.txt").read().split()):
    if rows[i][0] == "??":
        v = int(pc, 16)
        for a, b, o, path in maps:
            if a <= v < b:
                rows[i][0] = sym(path, v - a + o)
                break
# libc-internal samples (memset / memcpy ifuncs: not exported, shown as the preceding export): by caller
rets = open("pcs.txt.ret").read().split()
lib = [(i, r) for i, r in enumerate(rets) if not rows[i][0].startswith(("vvc", "(anon", "std", "bigbuf", "int ", "void ", "build", "plan", "valid"))]
if lib:
    res = subprocess.run(["addr2line", "-f", "-C", "-e", "host_prof"], input="\n".join(r for _, r in lib), capture_output=True, text=True).stdout.split("\n")
    cc = collections.Counter(res[2 * k][:100] for k in range(len(lib)))
    print("--- shared-library samples (%d) by return address" % len(lib))
    for f, c in cc.most_common(12):
        print("%5.1f%%  %s" % (100 * c / n, f))
for f, c in fn.most_common(25):
    print("%5.1f%%  %s" % (100 * c / n, f))
print("--- lines")
for f, c in ln.most_common(40):
    print("%5.1f%%  %s" % (100 * c / n, f))
EOF
else
  rm -f gmon.out && ./host_prof "../$1" "${2:-1}" && gprof -b -p host_prof gmon.out | head -45
fi
