"""CPU-tier guard for the host tier: ``tests/test_gpu_host.py`` calls CPU-tier
test functions directly, so a new ``parametrize`` argument on one of them
breaks the GPU tier only on the box. Check every such call passes as many
positional arguments as the callee takes."""

import ast
import inspect
import os
import sys

from conftest import ROOT


def _calls():
    tree = ast.parse(open(os.path.join(ROOT, "tests", "test_gpu_host.py")).read())
    for node in ast.walk(tree):
        if (isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute)
                and isinstance(node.func.value, ast.Name) and node.func.value.id.startswith("test_")
                and node.func.attr.startswith("test_")):
            yield node.func.value.id, node.func.attr, len(node.args) + len(node.keywords), node.lineno


def test_host_tier_calls_match_cpu_tier_signatures():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    seen = 0
    for mod_name, fn_name, nargs, line in _calls():
        fn = getattr(__import__(mod_name), fn_name)
        params = [p for p in inspect.signature(fn).parameters.values() if p.default is inspect.Parameter.empty]
        assert nargs == len(params), f"test_gpu_host.py:{line} calls {mod_name}.{fn_name} with {nargs} args, " \
                                     f"it takes {[p.name for p in params]}"
        seen += 1
    assert seen >= 10
