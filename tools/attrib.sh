#!/bin/bash
# Per-phase VALU attribution of the config-2 render kernel (VERDICT r4 "next" 2): one
# rocprofv3 PMC pass (SQ_INSTS_VALU, SQ_INSTS_SALU, SQ_WAVES) per library -- the product
# build and the SPT_DUP builds (spt_path.h: each runs one phase twice on opaque inputs and
# discards the copy) -- over the same short bench command; the difference in VALU per
# render launch is the duplicated phase's instruction count.
# Build first (build host): make -C simplepathtracer_amd/csrc variants \
#   VARIANTS="$(for b in 1 2 4 8 16 32 64 128; do echo -n "dup$b:-DSPT_DUP=$b "; done)"
# Usage (GPU box): tools/attrib.sh <tag> [lib ...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-attrib}
shift
LIBS="$*"
[ -z "$LIBS" ] && LIBS="libspt_hip.so $(for b in 1 2 4 8 16 32 64 128; do echo libspt_hip_dup$b.so; done)"
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for lib in $LIBS; do
  [ -f "$R/simplepathtracer_amd/lib/$lib" ] || { echo "missing $lib"; exit 3; }
  d="$OUT/${lib%.so}"
  mkdir -p "$d"
  echo "== $lib"
  SPT_LIB=$lib timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv \
    -d "$d" -o run -- python3 "$R/bench.py" ${ATTRIB_ARGS:---steps 4 --warmup 1} --no-cpu-baseline --no-dropin --service 0 \
    > "$d/log" 2>&1
  rc=$?
  echo "== $lib rc=$rc"
  case $rc in 0) ;; *) tail -n 5 "$d/log"; exit $rc ;; esac
done
python3 - "$OUT" $LIBS <<'PY'
import csv, glob, json, os, sys
out, libs = sys.argv[1], sys.argv[2:]
res = {}
for lib in libs:
    agg = {}
    for f in glob.glob(os.path.join(out, lib[:-3], "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "spt::render_kernel" in r["Kernel_Name"]:
                agg.setdefault(r["Counter_Name"], []).append((r.get("Dispatch_Id", ""), float(r["Counter_Value"])))
    # bench.py's one-row probe launch is a render_kernel dispatch too: frames only (VALU
    # above 1% of the largest dispatch's)
    big = {d for d, v in agg.get("SQ_INSTS_VALU", []) if v > 0.01 * max(x for _, x in agg["SQ_INSTS_VALU"])}
    agg = {c: [v for d, v in xs if d in big] for c, xs in agg.items()}
    res[lib] = {k: sum(v) / len(v) for k, v in agg.items()}
    res[lib]["launches"] = len(agg.get("SQ_INSTS_VALU", []))
base = res[libs[0]]
print(f"{'library':26s} {'VALU/launch':>16s} {'dVALU':>14s} {'SALU/launch':>16s} {'dSALU':>14s} launches")
for lib in libs:
    r = res[lib]
    print(f"{lib:26s} {r.get('SQ_INSTS_VALU', 0):16,.0f} {r.get('SQ_INSTS_VALU', 0) - base.get('SQ_INSTS_VALU', 0):14,.0f} "
          f"{r.get('SQ_INSTS_SALU', 0):16,.0f} {r.get('SQ_INSTS_SALU', 0) - base.get('SQ_INSTS_SALU', 0):14,.0f} {r['launches']}")
json.dump(res, open(os.path.join(out, "attrib.json"), "w"), indent=1)
PY
