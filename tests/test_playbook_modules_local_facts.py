"""The local executor gathers a host's node facts once for all of its sandboxes (executor.py)."""
from tritonk8ssupervisor_amd import executor as ex_mod
from tritonk8ssupervisor_amd.provider.base import Machine


def test_local_facts_are_gathered_once_per_ttl(monkeypatch):
    import tritonk8ssupervisor_amd.nodefacts as nf

    calls = []
    monkeypatch.setattr(nf, "node_facts", lambda timing=None: (calls.append(1), {"tk8s_host_gpus": len(calls)})[1])
    ms = {n: Machine(name=n, id=n, package="p", networks=[], primaryip="127.0.0.1", sandbox="/tmp") for n in ("a", "b")}
    ex = ex_mod.LocalExecutor(None, ms)
    a, b = ex.facts("a"), ex.facts("b")
    assert a == b == {"tk8s_host_gpus": 1} and len(calls) == 1
    a["x"] = 1  # callers get their own copy
    assert "x" not in ex.facts("a")
    monkeypatch.setattr(ex, "FACTS_TTL_S", -1.0)  # expired: gathered again
    assert ex.facts("b") == {"tk8s_host_gpus": 2}


def test_facts_gathering_reports_where_its_time_went():
    """The cold first run's slowest task was this gathering (0.33 s on a busy fresh box): its
    parts are timed into the task's event (timing_ms), so a slow one names its part."""
    import tritonk8ssupervisor_amd.nodefacts as nf

    timing: dict = {}
    facts = nf.node_facts(timing)
    assert "tk8s_rocm_version" in facts
    assert list(timing) == ["import", "rocm_version", "kfd_access", "gpu_inventory", "native_tools"]
    assert all(v >= 0 for v in timing.values())
    ms = {"a": Machine(name="a", id="a", package="p", networks=[], primaryip="127.0.0.1", sandbox="/tmp")}
    t2: dict = {}
    ex_mod.LocalExecutor(None, ms).facts("a", t2)
    assert "lock_wait" in t2 and "gpu_inventory" in t2


def test_rocm_version_comes_from_the_install_directory_name(tmp_path):
    """The cold first run's 0.8 s was the first read of .info/version on a fresh GPU box (its
    image pages files in on first read): the versioned directory's name is read instead."""
    from tritonk8ssupervisor_amd.nodefacts import rocm_version

    real = tmp_path / "rocm-7.2.0"
    (real / ".info").mkdir(parents=True)
    (real / ".info" / "version").write_text("should-not-be-read\n")
    (tmp_path / "rocm").symlink_to(real)
    assert rocm_version(tmp_path / "rocm") == "7.2.0"
    plain = tmp_path / "rocm-dev"
    (plain / ".info").mkdir(parents=True)
    (plain / ".info" / "version").write_text("6.4.1-120\n")
    assert rocm_version(plain) == "6.4.1-120"
    assert rocm_version(tmp_path / "missing") == ""
