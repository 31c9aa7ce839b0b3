set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 400 python3 -u tools/shard_profile.py --mode single --instances 50000 > $O/single50k.json 2> $O/single50k.err && tail -c 1500 $O/single50k.json &&
timeout -k 10 400 python3 -u tools/shard_profile.py --mode sharded --shards 2 --shared-stream > $O/sharded2.json 2> $O/sharded2.err && tail -c 3000 $O/sharded2.json &&
timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 > $O/bench_n2.log 2>&1 ; echo "bench n2 rc=$?"; tail -c 1500 $O/bench_n2.log
