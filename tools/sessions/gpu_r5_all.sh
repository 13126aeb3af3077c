#!/bin/bash
# Round 5: GPU tests + smoke, the comm-under-load A/B (legacy / node / native, reserved CUs), then the bench (N=1).
set -o pipefail
out=gpurun_out/${1:-r5g}
mkdir -p "$out"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
# where RCCL's start-up banner goes when the bench's ranks set NCCL_DEBUG=WARN + NCCL_DEBUG_FILE (stdout must hold
# only the JSON line)
NCCL_DEBUG=WARN NCCL_DEBUG_FILE="$PWD/$out/rccl_banner.%p.log" timeout -k 10 120 python -c "
import torch, torch.distributed as dist
dist.init_process_group('nccl', store=dist.HashStore(), rank=0, world_size=1, device_id=torch.device('cuda:0'))
t = torch.ones(4, device='cuda:0'); dist.all_reduce(t); torch.cuda.synchronize(); print('allreduce', t.tolist())
dist.destroy_process_group()" > "$out/rccl_banner.stdout" 2> "$out/rccl_banner.stderr" || exit $?
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$out/pytest.log" 2>&1 || exit $?
timeout -k 10 600 python -m otedama_amd.parallel.comm_probe --seconds 4 --windows 2 \
  --reserves "0;0,1,2,3,4,5,6,7;0,32,64,96,128,160,192,224" > "$out/comm.json" 2> "$out/comm.err" || exit $?
timeout -k 10 620 python bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
