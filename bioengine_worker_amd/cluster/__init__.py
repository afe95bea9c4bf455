"""Cluster runtime: node agent + resource accounting, SLURM autoscaling."""
