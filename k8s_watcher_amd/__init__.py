"""k8s-watcher-amd: a Kubernetes pod-event watcher with a native decode path.

Clean-room rebuild of highreso-gpu/k8s-watcher. Layers:

* ``utils``    — layered YAML config, log formats, backoff, timestamps (L1)
* ``net``      — asyncio HTTP/1.1 client shared by every link
* ``kube``     — kubeconfig / in-cluster auth and the core/v1 REST subset (L2a)
* ``models``   — attribute views over API JSON and the clusterapi payload
* ``ops``      — event decoding (C++ ``_kwcore`` or Python), filters, pod cache (L3)
* ``parallel`` — the clusterapi notifier pool and multi-process sharding (L2b)
* ``engine``   — reflector (list/watch/resume/410), pipeline, service, checkpoint (L4)
* ``compat``   — drop-in subset of the ``kubernetes`` client API
* ``testing``  — fake kube-apiserver, stub clusterapi, pod generator
"""

__version__ = "1.0.0"
