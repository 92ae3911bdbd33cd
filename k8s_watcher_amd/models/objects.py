"""Attribute-style views over raw Kubernetes JSON (stand-in for ``kubernetes.client.V1*``).

The reference's code reads pods as library model objects —
``pod.metadata.name``, ``pod.status.container_statuses[i].restart_count``,
``pod.metadata.creation_timestamp.isoformat()`` (``pod_watcher.py:159-202``).
This framework keeps pods as plain JSON dicts on the hot path and offers
:class:`ObjectView` for code that wants the library's attribute API:

* snake_case attributes map onto the API's camelCase keys
  (``container_statuses`` → ``containerStatuses``, ``pod_ip`` → ``podIP``);
* missing fields read as ``None`` (library models have every field);
* string-map fields (``labels``, ``annotations``, ...) stay plain dicts;
* known timestamp fields come back as tz-aware ``datetime`` objects;
* ``to_dict()`` gives the library's snake_case dict.

Views wrap without copying; construction cost is one object per accessed node.
"""

from __future__ import annotations

from typing import Any, Dict, Iterator

_SPECIAL = {
    "pod_ip": "podIP", "pod_ips": "podIPs", "host_ip": "hostIP", "host_ips": "hostIPs",
    "container_id": "containerID", "image_id": "imageID", "api_version": "apiVersion",
    "_continue": "continue", "_from": "from", "node_ip": "nodeIP", "cluster_ip": "clusterIP",
    "external_ip": "externalIP", "uid": "uid", "git_version": "gitVersion",
    "git_commit": "gitCommit", "git_tree_state": "gitTreeState", "build_date": "buildDate",
    "go_version": "goVersion",
}
_REVERSE_SPECIAL = {v: k for k, v in _SPECIAL.items()}

_MAP_FIELDS = frozenset({
    "labels", "annotations", "nodeSelector", "data", "binaryData", "capacity",
    "allocatable", "limits", "requests", "allocatedResources", "matchLabels",
    "stringData", "overhead", "selector_map",
})

_TIME_FIELDS = frozenset({
    "creationTimestamp", "deletionTimestamp", "startedAt", "finishedAt", "lastTransitionTime",
    "lastProbeTime", "startTime", "lastTimestamp", "firstTimestamp", "eventTime",
    "lastHeartbeatTime", "expirationTimestamp",
})


def snake_to_camel(name: str) -> str:
    special = _SPECIAL.get(name)
    if special is not None:
        return special
    head, *rest = name.split("_")
    return head + "".join(p[:1].upper() + p[1:] for p in rest)


def camel_to_snake(name: str) -> str:
    special = _REVERSE_SPECIAL.get(name)
    if special is not None:
        return special
    out = []
    for i, ch in enumerate(name):
        if ch.isupper() and i and not name[i - 1].isupper():
            out.append("_")
        out.append(ch.lower())
    return "".join(out)


def _wrap(key: str, value: Any) -> Any:
    if value is None:
        return None
    if key in _TIME_FIELDS and isinstance(value, str):
        from ..utils.timefmt import parse_k8s_time
        return parse_k8s_time(value)
    if isinstance(value, dict):
        if key in _MAP_FIELDS:
            return value
        return ObjectView(value)
    if isinstance(value, list):
        return [ObjectView(v) if isinstance(v, dict) else v for v in value]
    return value


class ObjectView:
    """Read-only attribute view over one JSON object."""

    __slots__ = ("_raw",)

    def __init__(self, raw: Dict[str, Any]) -> None:
        object.__setattr__(self, "_raw", raw if raw is not None else {})

    @property
    def raw(self) -> Dict[str, Any]:
        return self._raw

    def __getattr__(self, name: str) -> Any:
        if name.startswith("__"):
            raise AttributeError(name)
        key = snake_to_camel(name)
        return _wrap(key, self._raw.get(key))

    def __setattr__(self, name: str, value: Any) -> None:
        raise AttributeError("ObjectView is read-only")

    def __getitem__(self, key: str) -> Any:
        return self._raw[key]

    def get(self, key: str, default: Any = None) -> Any:
        return self._raw.get(key, default)

    def __iter__(self) -> Iterator[str]:
        return iter(self._raw)

    def __eq__(self, other: object) -> bool:
        if isinstance(other, ObjectView):
            return self._raw == other._raw
        return NotImplemented

    def __bool__(self) -> bool:
        # Library models are always truthy once present (SURVEY C8 relies on this).
        return True

    def to_dict(self) -> Dict[str, Any]:
        def conv(key: str, v: Any) -> Any:
            if isinstance(v, dict):
                if key in _MAP_FIELDS:
                    return dict(v)
                return {camel_to_snake(k): conv(k, x) for k, x in v.items()}
            if isinstance(v, list):
                return [conv(key, x) for x in v]
            if key in _TIME_FIELDS and isinstance(v, str):
                from ..utils.timefmt import parse_k8s_time
                return parse_k8s_time(v)
            return v
        return {camel_to_snake(k): conv(k, v) for k, v in self._raw.items()}

    def __repr__(self) -> str:
        import pprint
        return pprint.pformat(self.to_dict())


class ListView(ObjectView):
    """``*List`` response: ``.items`` is a list of views, ``.metadata`` the list meta."""

    __slots__ = ()


def as_view(obj: Any) -> Any:
    """Wrap a dict (no-op for views and non-dicts)."""
    if isinstance(obj, dict):
        return ObjectView(obj)
    return obj


def raw_of(obj: Any) -> Dict[str, Any]:
    """The JSON dict behind a view, a dict, or a library-style object with ``to_dict``."""
    if isinstance(obj, ObjectView):
        return obj.raw
    if isinstance(obj, dict):
        return obj
    to_dict = getattr(obj, "to_dict", None)
    if callable(to_dict):
        from .pod import snake_dict_to_api
        return snake_dict_to_api(to_dict())
    raise TypeError(f"cannot read a pod from {type(obj).__name__}")
