set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/split
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/split/t.log 2>&1 || { tail -30 gpurun_out/split/t.log; exit 1; }
tail -3 gpurun_out/split/t.log
timeout -k 10 200 python -u tools/bench_phase2.py > gpurun_out/split/b.log 2>&1
grep -v amdgpu.ids gpurun_out/split/b.log
