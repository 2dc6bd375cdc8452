#!/bin/bash
# the round-end GPU tier: every gpu-marked test in one process, then smoke()
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-fulltests}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -2 $O/smoke.log
