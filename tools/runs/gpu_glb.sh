set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/glb2
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_loci.py -k "phas or loci" -x -v --timeout 300 --timeout-method thread > gpurun_out/glb2/t.log 2>&1 || { tail -30 gpurun_out/glb2/t.log; exit 1; }
tail -3 gpurun_out/glb2/t.log
for args in "--samples 10000 --loci 200" "--samples 10000 --loci 200 --paired" "--samples 50000 --loci 16" "--samples 50000 --loci 16 --paired"; do
  echo "== $args" >> gpurun_out/glb2/b.log
  timeout -k 10 300 python -u tools/bench_loci.py $args --cpu-samples 200 --reps 2 >> gpurun_out/glb2/b.log 2>&1
done
grep -v amdgpu.ids gpurun_out/glb2/b.log | python -c "
import sys,json
for l in sys.stdin:
    l=l.strip()
    if l.startswith('=='): print(l)
    elif l.startswith('{'): d=json.loads(l); print(d['device_ms'], d['value'])
    else: print(l)"
