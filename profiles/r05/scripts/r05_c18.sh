#!/bin/bash
# Round 5, call 18: the driver's multi-GPU launch mode rehearsed on one GPU with
# this round's line (oracle_check on every N, the C5 sub-record): torch.distributed.run
# with 2 and 4 ranks, all on GPU 0 (--same-device: RCCL refuses a shared device,
# so the ranks agree on the P2P fallback), no other flags.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/${1:-r05_c18}
mkdir -p $O
for n in 2 4; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29517 + n)) bench.py --gpus $n --same-device --steps 20 --warmup 5 > $O/torchrun_$n.log 2>&1 \
    || { echo "n=$n rc=$?"; tail -20 $O/torchrun_$n.log; exit 3; }
  python3 -c "
import json
d=json.loads([l for l in open('$O/torchrun_$n.log') if l.startswith('{')][-1])
c5=d.get('c5_1024') or {}
print('n=$n', 'value %.4e'%d['value'], 'ms/step %.4f'%d['ms_per_step'], 'transport', d['config']['parallelism'], d.get('transport_fallback'))
print('  check', d['multi_rank_check'], 'oracle', d['oracle_check'])
print('  roofline', d['roofline'].get('bound'), d['roofline'].get('unit'), d['roofline'].get('frac'))
print('  c5', c5.get('value'), c5.get('ms_per_step'), c5.get('oracle_check', c5.get('error')))
"
done
