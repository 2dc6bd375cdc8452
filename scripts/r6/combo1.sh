bash scripts/r6/ipc.sh | tail -3 && bash scripts/r6/fsdp_ab.sh
