"""Loader and build driver for the native decoder extension ``_kwcore``.

The extension (``ops/csrc/kwcore.cpp``) is compiled in-tree with the host C++
compiler into ``k8s_watcher_amd/ops/_kwcore<EXT_SUFFIX>`` — by
``__graft_entry__.build()``, ``python -m k8s_watcher_amd.ops.native``, or
lazily by the test session. ``watcher.engine: native`` (the default) requires
it: :class:`NativeDecoder` raises :class:`NativeUnavailable` instead of
silently falling back to the Python engine.
"""

from __future__ import annotations

import importlib
import importlib.util
import os
import shutil
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "kwcore.cpp")
SO = os.path.join(HERE, "_kwcore" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))


class NativeUnavailable(ImportError):
    """The C++ extension is not built (run ``python -m k8s_watcher_amd.ops.native``)."""


def compiler() -> str:
    for cand in (os.environ.get("CXX"), "g++", "c++", "clang++"):
        if cand and shutil.which(cand):
            return cand
    raise NativeUnavailable("no C++ compiler found (set $CXX)")


SANITIZERS = {
    # host-code sanitizers for tests (scripts/sanitize.sh); never the production build
    "address": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
    "thread": ["-fsanitize=thread"],
}


def build_command(sanitize: str = "", out: str = SO) -> list:
    inc = sysconfig.get_paths()["include"]
    opt = ["-O1", "-g"] + SANITIZERS[sanitize] if sanitize else ["-O3"]
    return [compiler(), *opt, "-std=c++20", "-pthread", "-fPIC", "-shared", "-fvisibility=hidden",
            "-fno-strict-aliasing", "-Wall", "-Wno-shadow", "-Wno-unused-function", "-Wno-psabi",
            f"-I{inc}", f"-I{os.path.dirname(SRC)}", SRC, "-o", out, "-lssl", "-lcrypto", "-lz"]


def sanitizer_so(kind: str) -> str:
    """Path of the sanitizer build of the extension (outside the package: never imported by default)."""
    root = os.path.dirname(os.path.dirname(HERE))
    return os.path.join(root, "build", f"sanitize-{kind}", os.path.basename(SO))


def build_sanitized(kind: str, quiet: bool = False) -> str:
    """Compile ``_kwcore`` with ``-fsanitize=<kind>`` into ``build/sanitize-<kind>/``.

    Load it with ``$K8S_WATCHER_KWCORE_SO=<path>`` and the matching runtime in
    ``LD_PRELOAD`` (the interpreter itself is not instrumented).
    """
    out = sanitizer_so(kind)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = build_command(kind, out + ".tmp")
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise NativeUnavailable(f"building sanitized _kwcore failed:\n{' '.join(cmd)}\n{res.stderr}")
    os.replace(out + ".tmp", out)
    if not quiet:
        print(f"built {out}")
    return out


def sources() -> list:
    d = os.path.dirname(SRC)
    return [os.path.join(d, f) for f in sorted(os.listdir(d)) if f.endswith((".cpp", ".inc", ".h"))]


def is_fresh() -> bool:
    return os.path.exists(SO) and all(os.path.getmtime(SO) >= os.path.getmtime(s) for s in sources())


def build(quiet: bool = False) -> str:
    tmp = SO + ".tmp"
    cmd = build_command(out=tmp)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise NativeUnavailable(f"building _kwcore failed:\n{' '.join(cmd)}\n{res.stderr}")
    os.replace(tmp, SO)
    if not quiet:
        print(f"built {SO}")
    return SO


def ensure_built(quiet: bool = True) -> str:
    if not is_fresh():
        build(quiet)
    return SO


_mod = None


def load():
    global _mod
    if _mod is None:
        override = os.environ.get("K8S_WATCHER_KWCORE_SO")
        if override:  # a sanitizer build (build_sanitized); tests only
            spec = importlib.util.spec_from_file_location("k8s_watcher_amd.ops._kwcore", override)
            if spec is None or spec.loader is None:
                raise NativeUnavailable(f"cannot load {override}")
            mod = importlib.util.module_from_spec(spec)
            sys.modules["k8s_watcher_amd.ops._kwcore"] = mod
            spec.loader.exec_module(mod)
            _mod = mod
            return _mod
        try:
            _mod = importlib.import_module("k8s_watcher_amd.ops._kwcore")
        except ImportError as exc:
            raise NativeUnavailable(
                f"native engine requested but {os.path.basename(SO)} is not built ({exc}); "
                "run `python -m k8s_watcher_amd.ops.native` or set watcher.engine: python") from None
    return _mod


def available() -> bool:
    try:
        load()
        return True
    except NativeUnavailable:
        return False


class NativeDecoder:
    """Same interface as :class:`..decode.PyDecoder`, backed by ``_kwcore.StreamDecoder``."""

    name = "native"

    def __init__(self, environment: str, state_format: str = "structured", extra: int = 0,
                 validate: str = "payload") -> None:
        from .decode import VALIDATE_MODES
        mod = load()
        d = mod.StreamDecoder(environment, state_format)
        if extra:
            d.set_extra(extra)
        d.set_validate(VALIDATE_MODES[validate])
        if state_format == "python_repr":  # rendered natively (ops/csrc/pyrepr.inc), odd states by Python
            from ..models.payload import repr_fallback, utc_tzinfo_repr
            d.set_repr(utc_tzinfo_repr(), repr_fallback(environment, extra))
        self.extra = extra
        self._d = d
        self.environment = environment
        self.state_format = state_format
        # bind C methods directly: no Python frame per call
        self.feed = d.feed
        self.feed_chunked = d.feed_chunked
        self.body_done = d.body_done
        self.reset = d.reset
        self.decode_list = d.decode_list
        self.core = d.core
        self.core_from_summary = d.core_from_summary
        self.stats = d.stats


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] in SANITIZERS:
        build_sanitized(sys.argv[1])
        sys.exit(0)
    build(quiet=False)
    mod = load()
    print("loaded", mod.__file__, mod.cpu_features())
    sys.exit(0)
