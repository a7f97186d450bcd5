R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_lat2; mkdir -p $O; cd $R; export TMPDIR=/tmp KGPU_HOST_TRACE=1
for w in d:5000 d:100000 b:5000 c:5000; do cfg=${w%%:*}; n=${w##*:}
  timeout -k 10 300 python3 -u tools/latency_probe.py --config $cfg --nodes $n --pods 300 > $O/lat_${cfg}${n}.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_schedule_one.py tests/test_prepare_pods.py tests/test_topo_persistent.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
