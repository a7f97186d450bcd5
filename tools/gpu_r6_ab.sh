R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_ab1; mkdir -p $O; cd $R; export TMPDIR=/tmp
for v in a b; do
  KGPU_LIB_PATH=$R/kubernetes-1_amd/kgpu/libkgpu_$v.so timeout -k 10 400 python -u -m pytest tests/test_full_size.py tests/test_pipeline.py tests/test_batch_helper.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || exit 1
done
bash tools/gpu_ab3.sh r06_ab1 b:5000 3
