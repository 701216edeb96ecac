#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_embedding_known_answers_gpu.py tests/test_gpu_parity.py -k "embed or matches_reference or width" > gpurun_out/embed_tests.log 2>&1
rc=$?; tail -2 gpurun_out/embed_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --roofline-only --no-cpu-baseline > gpurun_out/roof.log 2>&1
rc=$?; python3 -c "
import json
for l in open('gpurun_out/roof.log'):
    if l.startswith('{'):
        d=json.loads(l)
        for e in [d.get('roofline')]+d.get('roofline_aux',[]):
            print(e['kernel'], e['avg_ms'], e['achieved'], e['unit'], e['frac'])
"; exit $rc
