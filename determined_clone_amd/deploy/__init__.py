"""Cluster deployment helpers (reference: `harness/determined/deploy/`)."""
