set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ph
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "phasing" -x -v --timeout 120 --timeout-method thread > gpurun_out/ph/t.log 2>&1 || { tail -30 gpurun_out/ph/t.log; exit 1; }
tail -3 gpurun_out/ph/t.log
timeout -k 10 300 python -u tools/bench_phase2.py > gpurun_out/ph/b.log 2>&1
cat gpurun_out/ph/b.log | grep -v amdgpu.ids
