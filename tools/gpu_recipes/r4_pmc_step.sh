# Hardware counters of the one-client Intrusion step (microbench --step-only) (rocprofv3 --pmc, one pass per counter group,
# kernels filtered by name), then per-kernel means of every counter.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4pmcstep}
mkdir -p $O
cd /tmp
P="python3 $R/tools/microbench.py --step-only"
K="."
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES" \
           "SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd $R && timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "$K" --output-format csv -d $O/p$i -o run -- $P > $O/p$i.log 2>&1) || exit 1
done
python3 - $O <<'PY' > $O/pmc_means.txt
import collections, csv, glob, os, sys
per = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(os.path.join(sys.argv[1], "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(path)):
        name = row.get("Kernel_Name", "?").split("(")[0].replace("void ", "").replace("fedtgan::", "")
        per[f"{name[:60]} grid={row.get('Grid_Size', '?')}"][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in sorted(per.items()):
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
PY
rm -rf $O/p1 $O/p2 $O/p3 $O/p4
echo done
