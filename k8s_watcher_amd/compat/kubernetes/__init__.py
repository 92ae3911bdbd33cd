"""Drop-in subset of the ``kubernetes`` Python client.

``from k8s_watcher_amd.compat.kubernetes import client, config, watch`` gives
the calls the reference makes without the (unavailable) library. See the
module docstrings for the exact surface.
"""

from . import client, config, watch  # noqa: F401

__all__ = ["client", "config", "watch"]
