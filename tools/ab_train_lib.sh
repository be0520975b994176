cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "f32 or config5 or sg_f32" > gpurun_out/pytest_abt.log 2>&1 || { tail -20 gpurun_out/pytest_abt.log; exit 1; }
tail -2 gpurun_out/pytest_abt.log
for i in 1 2; do
  for v in A B; do
    lib=build/lib_base.so; [ $v = B ] && lib=sg-nerf_amd/libsgn_hip.so
    SGN_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 200 python bench.py --train --steps 40 --warmup 5 > gpurun_out/abt_$v$i.json 2> gpurun_out/abt_$v$i.err || { tail -5 gpurun_out/abt_$v$i.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/abt_$v$i.json')); print('$v', round(d['ms_per_step'],3))"
  done
done
