set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lsplit
for args in "--samples 3202" "--samples 3202 --paired" "--samples 1000" "--samples 1000 --paired"; do
  echo "== $args" >> gpurun_out/lsplit/b.log
  timeout -k 10 300 python -u tools/bench_loci.py $args --cpu-samples 200 --reps 2 >> gpurun_out/lsplit/b.log 2>&1
done
grep -v amdgpu.ids gpurun_out/lsplit/b.log
