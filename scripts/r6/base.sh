# round-6 baseline on a fresh box: headline bench + isolated attention timing
set -o pipefail
OUT=gpurun_out/r6base; mkdir -p $OUT
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/bench1.json 2> $OUT/bench1.err && \
timeout -k 10 300 python3 tools/attn_ab.py --rounds 5 > $OUT/attn.jsonl 2> $OUT/attn.err && \
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?; cat $OUT/bench1.json $OUT/attn.jsonl $OUT/bench2.json; exit $rc
