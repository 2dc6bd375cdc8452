#!/bin/bash
cd $GRAFT_REPO_ROOT
bash scripts/r5/final.sh r5final || exit $?
bash scripts/r5/prio_ab.sh r5prio
