set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 400 python3 -u tools/shard_profile.py --mode sharded --shards 2 --shared-stream > $O/sharded2.json 2> $O/sharded2.err && tail -c 3000 $O/sharded2.json &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --no-beside --warmup 15 > $O/bench1.log 2>&1 && tail -c 600 $O/bench1.log &&
timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_n2.log 2>&1 ; echo "bench n2 rc=$?"; tail -c 1200 $O/bench_n2.log
