"""Operator tools (capture a cluster's pod stream for offline replay)."""
