#!/bin/bash
# offload tests (incl. proxy-mode gathers) + 70B proxy-8 offload runs + BasicLLM job kernel trace
cd $GRAFT_REPO_ROOT
OFF_OUT=r5off70b bash scripts/r5/batch3.sh r5batch4 || exit $?
bash scripts/r5/basicllm_prof.sh r5basicllm
