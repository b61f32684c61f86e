# Persistent-kernel probe, round 4: two-level XCD barrier + real cross-boundary data vs a graph of kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4persist}
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/persistent_probe2 $R/csrc/probes/persistent_probe2.hip || exit 1
timeout -k 10 60 /tmp/persistent_probe2 25 200 > $OUT/probe.txt 2>&1 || exit 1
timeout -k 10 60 /tmp/persistent_probe2 8 200 >> $OUT/probe.txt 2>&1 || exit 1
echo done
