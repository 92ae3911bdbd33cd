"""Config loader against the §5.6 effective-config table."""

import os

import pytest

from k8s_watcher_amd.utils.config import (ConfigError, deep_merge, load_config_file, load_layered_config,
                                          load_settings, parse_override, settings_from_dict, substitute_env)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(ROOT, "config")


def test_deep_merge_override_wins_and_lists_replace():
    base = {"a": {"x": 1, "y": [1, 2]}, "b": 1}
    over = {"a": {"y": [3], "z": 2}, "c": 3}
    out = deep_merge(base, over)
    assert out == {"a": {"x": 1, "y": [3], "z": 2}, "b": 1, "c": 3}
    # inputs untouched (deep copy)
    assert base == {"a": {"x": 1, "y": [1, 2]}, "b": 1}


def test_deep_merge_dict_replaced_by_scalar():
    assert deep_merge({"a": {"x": 1}}, {"a": None}) == {"a": None}


def test_substitute_whole_string_only():
    env = {"K": "v", "EMPTY": ""}
    doc = {"a": "${K}", "b": "${MISSING}", "c": "${MISSING:-dflt}", "d": "x${K}",
           "e": ["${K}", {"f": "${K:-z}"}], "g": 5, "h": "${EMPTY:-d}"}
    out = substitute_env(doc, env)
    assert out == {"a": "v", "b": "", "c": "dflt", "d": "x${K}", "e": ["v", {"f": "v"}], "g": 5, "h": ""}


def test_default_containing_separator():
    assert substitute_env("${A:-x:-y}", {}) == "x:-y"


def test_missing_and_empty_files(tmp_path, capsys):
    assert load_config_file(str(tmp_path / "nope.yaml")) == {}
    assert "not found" in capsys.readouterr().out
    (tmp_path / "empty.yaml").write_text("")
    assert load_config_file(str(tmp_path / "empty.yaml")) == {}
    (tmp_path / "bad.yaml").write_text("a: [1,\n")
    assert load_config_file(str(tmp_path / "bad.yaml")) == {}
    assert "Error loading config" in capsys.readouterr().out


@pytest.mark.parametrize("env,level,namespaces,critical,incluster,config_file", [
    ("development", "DEBUG", ["default", "kube-system"], False, False, "./assets/config"),
    ("staging", "INFO", [], False, False, None),
    ("production", "WARNING", ["default", "production", "monitoring", "kube-system"], True, True, None),
])
def test_effective_config_table(env, level, namespaces, critical, incluster, config_file):
    """SURVEY §5.6 effective-config table, recomputed from the shipped YAML."""
    s = load_settings(env, CFG, environ={})
    assert s.watcher.log_level == level
    assert s.watcher.namespaces == namespaces
    assert s.watcher.critical_events_only is critical
    assert s.kubernetes.use_incluster_config is incluster
    assert s.kubernetes.config_file == config_file
    assert s.clusterapi.timeout == 30
    assert s.clusterapi.pod_update == "/api/pods/update"
    assert s.clusterapi.health == "/health"
    assert s.clusterapi.retry.max_attempts == 3
    assert s.clusterapi.retry.delay_seconds == 2
    assert s.clusterapi.api_key == ""


def test_clusterapi_base_urls():
    assert load_settings("development", CFG, environ={}).clusterapi.base_url == "http://localhost:3000"
    assert load_settings("staging", CFG, environ={}).clusterapi.base_url == "http://localhost:3000"
    assert load_settings("production", CFG, environ={}).clusterapi.base_url == "https://prod-clusterapi.example.com"


def test_api_key_from_environment():
    s = load_settings("production", CFG, environ={"PROD_CLUSTERAPI_API_KEY": "sekret"})
    assert s.clusterapi.api_key == "sekret"
    s = load_settings("development", CFG, environ={"CLUSTERAPI_API_KEY": "dev"})
    assert s.clusterapi.api_key == "dev"


def test_top_level_environment_key_kept_but_unused():
    raw = load_layered_config("development", CFG, environ={})
    assert raw["environment"] == "local"
    assert load_settings("development", CFG, environ={}).environment == "development"


def test_invalid_values_raise():
    with pytest.raises(ConfigError):
        settings_from_dict("staging", {"watcher": {"log_level": "LOUD"}})
    with pytest.raises(ConfigError):
        settings_from_dict("staging", {"watcher": {"notify_on": "sometimes"}})
    with pytest.raises(ConfigError):
        settings_from_dict("staging", {"watcher": {"namespaces": "default"}})
    with pytest.raises(ConfigError):
        settings_from_dict("staging", {"clusterapi": {"timeout": "soon"}})


def test_overrides():
    ov = deep_merge(parse_override("watcher.notify_on=phase_change"),
                    parse_override("clusterapi.pool.connections=4"))
    s = load_settings("staging", CFG, overrides=ov, environ={})
    assert s.watcher.notify_on == "phase_change"
    assert s.clusterapi.pool.connections == 4
    with pytest.raises(ConfigError):
        parse_override("novalue")


def test_config_dir_fallback_when_cwd_has_no_config(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    monkeypatch.delenv("K8S_WATCHER_CONFIG_DIR", raising=False)
    s = load_settings("production", environ={})
    assert s.watcher.critical_events_only is True


def test_config_dir_env_override(tmp_path, monkeypatch):
    (tmp_path / "base.yaml").write_text("watcher:\n  log_level: ERROR\n")
    (tmp_path / "staging.yaml").write_text("")
    monkeypatch.setenv("K8S_WATCHER_CONFIG_DIR", str(tmp_path))
    assert load_settings("staging", environ={}).watcher.log_level == "ERROR"


def test_retry_policy_delays():
    s = load_settings("staging", CFG, environ={})
    r = s.watcher.retry
    assert [r.delay(i) for i in (1, 2, 3)] == [5, 10, 20]
    assert r.delay(100) == r.max_delay_seconds


def test_retired_keys_load_with_a_warning(caplog):
    """Settings retired in round 6 (fixed at their measured winner) still load
    from an operator's file: ignored, each named in a warning; the reference's
    watch_interval is accepted silently."""
    import logging

    from k8s_watcher_amd.utils.config import load_settings, retired_keys_in
    ov = {"watcher": {"hub_framing": "on", "gc_freeze": False, "watch_interval": 3,
                      "leader_election": {"release_on_shutdown": False}},
          "clusterapi": {"pool": {"io_thread_on_rate": 10}, "spool": {"replay_batch": 5}}}
    with caplog.at_level(logging.WARNING, logger="k8s_watcher_amd.config"):
        s = load_settings("production", overrides=ov, environ={})
    named = sorted(retired_keys_in(s.raw))
    assert named == ["clusterapi.pool.io_thread_on_rate", "clusterapi.spool.replay_batch", "watcher.gc_freeze",
                     "watcher.hub_framing", "watcher.leader_election.release_on_shutdown"]
    text = caplog.text
    assert all(k in text for k in named) and "watch_interval" not in text
    assert s.clusterapi.pool.io_thread == "auto"
    assert load_settings("production", overrides={"clusterapi": {"pool": {"io_thread": True}}},
                         environ={}).clusterapi.pool.io_thread == "on"
