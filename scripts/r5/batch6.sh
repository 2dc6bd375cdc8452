#!/bin/bash
cd $GRAFT_REPO_ROOT
bash scripts/r5/hostlink.sh r5hostlink || exit $?
bash scripts/r5/basicllm_prof.sh r5basicllm || exit $?
bash scripts/r5/offtrace.sh r5offtrace
