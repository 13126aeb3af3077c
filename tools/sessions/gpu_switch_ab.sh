#!/bin/bash
# Job switches and rates of the host-stored abort word (vs the control stream), the X11 stage polls + per-slot digest buffers, the scrypt write-loop scalar polls and the staggered scrypt halves, each
# against the round-3 behaviour (env B) in the same session. Every GPU step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/switch_ab
mkdir -p $D
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
OLD_X11=OTEDAMA_X11_MIDPOLL=0,OTEDAMA_X11_OVERLAP=0
timeout -k 10 360 python tools/switch_ab.py --algo sha256d --env-b OTEDAMA_HOST_ABORT=0 > $D/switch_sha256d.jsonl 2> $D/switch_sha256d.err && cat $D/switch_sha256d.jsonl &&
timeout -k 10 300 python tools/ab_miner.py --a . --b . --algo sha256d --rounds 4 --seconds 6 --env-b OTEDAMA_HOST_ABORT=0 > $D/ab_sha256d.json 2> $D/ab_sha256d.err && cat $D/ab_sha256d.json &&
timeout -k 10 360 python tools/switch_ab.py --algo x11 --env-b $OLD_X11 > $D/switch_x11.jsonl 2> $D/switch_x11.err && cat $D/switch_x11.jsonl &&
timeout -k 10 360 python tools/switch_ab.py --algo scrypt --env-b OTEDAMA_SCRYPT_POLL=0 > $D/switch_scrypt.jsonl 2> $D/switch_scrypt.err && cat $D/switch_scrypt.jsonl &&
timeout -k 10 360 python tools/switch_ab.py --algo scrypt --env-b OTEDAMA_SCRYPT_POLL=0,OTEDAMA_SCRYPT_HALVES=0 > $D/switch_scrypt_r3.jsonl 2> $D/switch_scrypt_r3.err && cat $D/switch_scrypt_r3.jsonl &&
timeout -k 10 400 python tools/ab_miner.py --a . --b . --algo scrypt --rounds 4 --seconds 8 --env-b OTEDAMA_SCRYPT_POLL=0 > $D/ab_scrypt_poll.json 2> $D/ab_scrypt_poll.err && cat $D/ab_scrypt_poll.json &&
timeout -k 10 300 python tools/ab_miner.py --a . --b . --algo x11 --rounds 4 --seconds 6 --env-b $OLD_X11 > $D/ab_x11.json 2> $D/ab_x11.err && cat $D/ab_x11.json &&
timeout -k 10 400 python tools/ab_miner.py --a . --b . --algo scrypt --rounds 4 --seconds 8 --env-b OTEDAMA_SCRYPT_HALVES=0 > $D/ab_scrypt.json 2> $D/ab_scrypt.err && cat $D/ab_scrypt.json
