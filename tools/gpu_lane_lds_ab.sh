# dp_lane_kernel hand-off A/B on cfg5 full DP (indel -2): LDS 4-bit steps (default) vs int16 column in HBM
# (OVL_LANE_LDS=0) vs the previous build; lane parity tests first, then FETCH/WRITE passes for both forms.
set -u
cd "$GRAFT_REPO_ROOT"
P=$GRAFT_REPO_ROOT/genome-assembly-using-overlap-graphs_amd
OUT=$GRAFT_REPO_ROOT/gpurun_out/lds
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dp_lane.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1; rc=$?
tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
run() {  # tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --config cfg5 --indel -2 --steps 20 --warmup 3 --no-extra --no-cpu-baseline > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail -5 "$OUT/$tag.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'kernel_ms %.3f step_ms %.3f' % (d['roofline']['kernel_ms'], d['ms_per_step']))" "$OUT/$tag.json" $tag
}
for rep in 1 2; do
  run lds OVL_LIB_PATH=$P/build/libovl.so
  run hbm16 OVL_LIB_PATH=$P/build/libovl.so OVL_LANE_LDS=0
  run old OVL_LIB_PATH=$P/build/ab_old/libovl.so
done
for form in lds hbm16; do
  [ $form = hbm16 ] && export OVL_LANE_LDS=0
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -T --kernel-include-regex dp_lane_kernel -d "$OUT/$form-$ctr" -o p --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config cfg5 --indel -2 --steps 5 --warmup 1 --no-cpu-baseline --no-extra > "$OUT/$form-$ctr.log" 2>&1 || { echo "pmc $form $ctr failed"; tail -20 "$OUT/$form-$ctr.log"; exit 1; }
  done
  python3 - "$OUT" $form <<'PY'
import csv, glob, sys, os
out, form = sys.argv[1], sys.argv[2]
vals = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(os.path.join(out, f"{form}-{ctr}", "**", "*counter_collection.csv"), recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == ctr]
    per = {}
    for r in rows:
        per.setdefault(r["Dispatch_Id"], 0.0)
        per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    vals[ctr] = sum(per.values()) / len(per)
hbm = (2 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024
print(form, "FETCH_SIZE", vals["FETCH_SIZE"], "WRITE_SIZE", vals["WRITE_SIZE"], "hbm_bytes_per_launch %.4g" % hbm)
PY
done
unset OVL_LANE_LDS
