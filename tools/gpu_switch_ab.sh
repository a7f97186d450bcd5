#!/bin/bash
# GPU call: alternated bench runs of the in-tree build under engine switches (bench.py flags), R rounds.
#   tools/gpu_switch_ab.sh <out-name> "<cfg:nodes ...>" <rounds> "<label>=<bench flags>" ...
# e.g. tools/gpu_switch_ab.sh r06_sw "c:100000" 3 "base=" "nosleep=--tbatch-poll-sleep 0"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-switch_ab}
WL=${2:-c:5000}
N=${3:-3}
shift 3
mkdir -p $O
cd $R && export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc" >> $O/status.txt; return $rc; }
for w in $WL; do
  cfg=${w%%:*}; n=${w##*:}
  for r in $(seq 1 $N); do
    for v in "$@"; do
      label=${v%%=*}; flags=${v#*=}
      step ab_${cfg}${n}_${label}_$r timeout -k 10 300 python3 -u bench.py --config $cfg --nodes $n --steps 10 --warmup 2 \
        --cpu-sample 0 --latency-pods 0 --dropin-pods 0 --extender-pods 0 --extras "" $flags || exit 1
    done
  done
done
