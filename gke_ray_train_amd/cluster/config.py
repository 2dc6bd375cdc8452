"""Address resolution for the node-local cluster (``ray.init(address=...)`` compatibility)."""
from __future__ import annotations

import os


def resolve_address(address: str) -> str:
    """Accept the reference's address forms; everything resolves to this node.

    ``http://localhost:8265`` (the job-server address the reference port-forwards to,
    a3-mega/gke-ray-cluster-setup.sh:68-71) and ``host:6379`` GCS addresses are accepted as long
    as the host is local: there is one node.
    """
    a = address.replace("http://", "").replace("https://", "").replace("ray://", "")
    host = a.split(":")[0]
    if host not in ("localhost", "127.0.0.1", "0.0.0.0", os.uname().nodename, ""):
        raise ConnectionError(f"{address}: only the local node is supported by this runtime")
    return "local"
