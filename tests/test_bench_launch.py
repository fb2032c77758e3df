"""bench.py's rank launcher (CPU): `python bench.py --gpus N` outside a
torch.distributed launch must start N rank processes (one per GPU, the
reference's Lightning DDP over all devices, main.py:108-119) before anything
touches the GPU; under torchrun, WORLD_SIZE must equal --gpus."""
import importlib.util
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_single_gpu_runs_in_process():
    b = _bench()
    assert b.launch_plan([], {}) is None
    assert b.launch_plan(["--gpus", "1", "--steps", "2"], {}) is None


def test_multi_gpu_spawns_ranks():
    b = _bench()
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "2"]
    cmd = b.launch_plan(argv, {})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert any(c.startswith("--master-port=") and int(c.split("=")[1]) > 0 for c in cmd)
    assert cmd[-len(argv) - 1] == os.path.join(REPO, "bench.py")
    assert cmd[-len(argv):] == argv  # the ranks see the same --gpus and see WORLD_SIZE


def test_ranks_under_torchrun_run_in_process():
    b = _bench()
    assert b.launch_plan(["--gpus", "4"], {"WORLD_SIZE": "4"}) is None


def test_world_size_mismatch_refused():
    b = _bench()
    with pytest.raises(SystemExit) as e:
        b.launch_plan(["--gpus", "8"], {"WORLD_SIZE": "2"})
    assert e.value.code == 2
    # end to end: refused before torch or the package is imported
    env = dict(os.environ, WORLD_SIZE="1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "refusing" in r.stderr


def test_launcher_starts_children_and_returns_their_status(tmp_path):
    """The launch path never imports torch in the parent: a fake
    torch.distributed.run on PYTHONPATH records its argv and exits 3; bench.py
    must exit with that status."""
    pkg = tmp_path / "torch" / "distributed"
    pkg.mkdir(parents=True)
    (tmp_path / "torch" / "__init__.py").write_text("")
    (pkg / "__init__.py").write_text("")
    rec = tmp_path / "argv.txt"
    (pkg / "run.py").write_text(f"import sys\nopen({str(rec)!r}, 'w').write(' '.join(sys.argv[1:]))\n"
                                "sys.exit(3)\n")
    env = dict(os.environ, PYTHONPATH=str(tmp_path))
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 3, r.stderr
    got = rec.read_text()
    assert "--nproc-per-node=2" in got and got.endswith("--gpus 2 --steps 1")


def test_pmc_fields_tied_to_kernel_sources(tmp_path, monkeypatch):
    """a committed PMC record's counters are printed only while
    the kernel's sources are the ones it was collected on (buildinfo digest);
    otherwise load_pmc returns None with the reason."""
    import json
    b = _bench()
    from tmr_amd import buildinfo
    rec = {"hbm_bytes_per_launch": 1.0, "source_digest": buildinfo.source_digest("heads")}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"round": "t", "configs": {"B": {"heads": rec}}}))
    monkeypatch.setattr(b, "PMC_FILE", str(p))
    got, why = b.load_pmc("B", "heads")
    assert why is None and got["hbm_bytes_per_launch"] == 1.0 and "round t" in got["source"]
    rec["source_digest"] = "0" * 16
    p.write_text(json.dumps({"round": "t", "configs": {"B": {"heads": rec}}}))
    got, why = b.load_pmc("B", "heads")
    assert got is None and "other kernel sources" in why
    assert b.load_pmc("C", "heads") == (None, "no PMC record for this config")


def test_source_digest_ignores_comments_only():
    """The digest hashes the code: a comment or layout edit keeps it, any
    token change moves it."""
    from tmr_amd import buildinfo
    a = b"int f(int x) { // twice\n  return 2 * x; /* doubled */ }\n"
    assert buildinfo._code("k.hip", a) == buildinfo._code("k.hip", b"int f(int x) {\n return 2 * x; }")
    assert buildinfo._code("k.hip", a) != buildinfo._code("k.hip", a.replace(b"2 * x", b"3 * x"))
    mk = b"# flags\nHIPFLAGS = -O3\n"
    assert buildinfo._code("Makefile", mk) == buildinfo._code("Makefile", b"HIPFLAGS = -O3")
    assert buildinfo._code("Makefile", mk) != buildinfo._code("Makefile", b"HIPFLAGS = -O2")


def test_committed_pmc_records_match_this_tree():
    """Every record of the committed profiles/pmc_by_config.json was collected
    on the kernel sources of this tree (so every bench line's traffic /
    mfma_busy_pmc is live): a kernel edit without re-running
    profiles/gpu_pmc.sh turns this red."""
    import json
    from tmr_amd import buildinfo
    d = json.load(open(os.path.join(REPO, "profiles", "pmc_by_config.json")))
    stale = []
    for cfg, roles in d["configs"].items():
        for role, rec in roles.items():
            if isinstance(rec, dict) and rec.get("source_digest") != buildinfo.source_digest(role):
                stale.append(f"{cfg}/{role}")
    assert set(d["configs"]) >= {"A", "B", "C", "D", "E"}
    assert not stale, f"PMC records from other kernel sources: {stale} (re-run profiles/gpu_pmc.sh)"


def test_frac_guard_nulls_fractions_above_one():
    b = _bench()
    out = {"roofline": {"frac": 0.2, "executed_frac": 1.3, "nested": {"x_frac": 2.0, "n": 5}}, "frac": 0.9}
    hits = b.guard_fracs(out)
    assert out["roofline"]["executed_frac"] is None and out["roofline"]["nested"]["x_frac"] is None
    assert out["roofline"]["frac"] == 0.2 and out["frac"] == 0.9 and out["roofline"]["nested"]["n"] == 5
    assert sorted(hits) == ["roofline.executed_frac=1.3", "roofline.nested.x_frac=2.0"]
