#!/bin/bash
# HBM traffic of every bench leg's kernels on THIS build, for the traffic
# index bench.py reads (profiles/<index>, tools/traffic_index.py): per leg,
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes over
# tools/cfg_time.py LEG (MI355X_MICROARCH.md "HBM": the two do not fit one TCC
# pass), each pass under its own limit, stopping at the first failure.
# tools/pmc_summary.py then gives per-kernel means per dispatch. The library's
# build stamp (kry_build_id) is written beside them, so an index entry is
# used only while the library it describes is the one loaded.
#   tools/pmc_legs.sh LEG[:STEPS] ...      -> gpurun_out/pmc_legs/LEG/summary.json, build_id
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_legs
mkdir -p "$OUT"
python3 -c "import sys; sys.path.insert(0, '.'); from krylov_amd import _lib; print(_lib.build_id())" > "$OUT/build_id" || exit 1
echo "build $(cat "$OUT/build_id")"
for spec in "$@"; do
  leg=${spec%%:*}; steps=""; [ "$leg" != "$spec" ] && steps=${spec#*:}
  mkdir -p "$OUT/$leg"
  i=0
  for c in FETCH_SIZE WRITE_SIZE; do
    i=$((i + 1))
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/$leg/p$i" \
      -o run -- python3 "$GRAFT_REPO_ROOT/tools/cfg_time.py" $leg $steps > "$OUT/$leg/p$i.log" 2>&1)
    rc=$?; echo "$leg $c rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/$leg/p$i.log"; exit $rc; }
  done
  python3 tools/pmc_summary.py "$OUT/$leg" > "$OUT/$leg/summary.json" || exit 1
done
exit 0
