# Round 6: does ANY torch-ROCm process exit 139 under rocprofv3 --kernel-trace on this image? (profiles/exit_r6.txt)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6l
mkdir -p $OUT
cd /tmp
run() {
  local n=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/$n -o run -- "$@" > $OUT/$n.log 2>&1
  echo "$n: exit $?" >> $OUT/exit.txt
  rm -rf $OUT/$n
}
run torch_sum python3 -c "import torch; x = torch.ones(1000, device='cuda'); print(float(x.sum()))"
run torch_matmul python3 -c "import torch; a = torch.randn(512, 512, device='cuda'); print(float((a @ a).sum()))"
run torch_graph python3 -c "import torch; x = torch.ones(1000, device='cuda'); g = torch.cuda.CUDAGraph(); s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s): y = x * 2
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g): y = x * 2
g.replay(); torch.cuda.synchronize(); print(float(y.sum()))"
cd $R
run ours_smoke python3 -c "import __graft_entry__ as e; e.smoke()"
echo done
