"""Single-node cluster bring-up (replaces the reference's GKE/KubeRay scripts and RayCluster CRs)."""
