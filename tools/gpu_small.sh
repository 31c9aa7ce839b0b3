set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/small
for n in 100000 12500; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --instances $n --steps 30 --warmup 20 > gpurun_out/small/b$n.log 2>&1 || { echo FAIL $n; tail -5 gpurun_out/small/b$n.log; exit 1; }
  grep '^{' gpurun_out/small/b$n.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
busy=sum(v['avg_us']*v['launches'] for v in d['kernels_probe'].values())/10
print('$n', 'value %.3e ms/step %.4f busy/step(us) %.1f' % (d['value'], d['ms_per_step'], busy))"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 10 --no-cpu-baseline > gpurun_out/small/r2.log 2>&1 || { echo R2FAIL; tail -5 gpurun_out/small/r2.log; exit 1; }
grep '^{' gpurun_out/small/r2.log | cut -c1-300
