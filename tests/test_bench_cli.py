"""bench.py's launch contract on the CPU (no GPU is touched by anything tested here).

* `--gpus N` decides the world: N rank processes are spawned when no launcher set WORLD_SIZE,
  a launcher's WORLD_SIZE must agree with --gpus, and a mismatch is refused (non-zero exit)
  instead of measuring one GPU under an N-GPU label (Missing 1).
* the PMC record feeds the bench line only for the library it measured (sha256 stamp).
"""

from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_rank_plan():
    assert bench.rank_plan(1, {}) == ("run", "")
    assert bench.rank_plan(4, {}) == ("spawn", "")
    assert bench.rank_plan(4, {"WORLD_SIZE": "4"}) == ("run", "")
    assert bench.rank_plan(1, {"WORLD_SIZE": "1"}) == ("run", "")
    plan, why = bench.rank_plan(8, {"WORLD_SIZE": "1"})
    assert plan == "refuse" and "WORLD_SIZE=1" in why
    assert bench.rank_plan(1, {"WORLD_SIZE": "2"})[0] == "refuse"
    assert bench.rank_plan(0, {})[0] == "refuse"


def test_gpu_count_is_distinct_devices():
    """n_gpus counts physical devices, not ranks (Weak 5): two ranks on one PCI
    address are one GPU with two ranks per device; one rank is unchanged."""
    one = [{"rank": 0, "device": 0, "pci": "0000:d9:00"}]
    assert bench.gpu_count(one) == (1, 1)
    shared = [{"rank": 0, "device": 0, "pci": "0000:d9:00"}, {"rank": 1, "device": 0, "pci": "0000:d9:00"}]
    assert bench.gpu_count(shared) == (1, 2)
    two = [{"rank": 0, "device": 0, "pci": "0000:0a:00"}, {"rank": 1, "device": 1, "pci": "0000:1a:00"}]
    assert bench.gpu_count(two) == (2, 1)


def test_spawn_ranks_environment(tmp_path):
    """Each spawned rank gets its own RANK / LOCAL_RANK, the common WORLD_SIZE and one port."""
    probe = tmp_path / "probe.py"
    out = tmp_path / "ranks"
    out.mkdir()
    probe.write_text(
        "import json, os, sys\n"
        f"d = {{k: os.environ.get(k) for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')}}\n"
        f"open(os.path.join({str(out)!r}, d['RANK'] + '.json'), 'w').write(json.dumps(d))\n"
        "sys.exit(0)\n")
    rc = bench.spawn_ranks(3, ["--steps", "5"], poll_s=0.05, script=str(probe))
    assert rc == 0
    rows = [json.loads((out / f"{r}.json").read_text()) for r in range(3)]
    assert [r["RANK"] for r in rows] == ["0", "1", "2"]
    assert [r["LOCAL_RANK"] for r in rows] == ["0", "1", "2"]
    assert {r["WORLD_SIZE"] for r in rows} == {"3"}
    assert {r["MASTER_ADDR"] for r in rows} == {"127.0.0.1"}
    assert len({r["MASTER_PORT"] for r in rows}) == 1


def test_spawn_ranks_failure_ends_the_others(tmp_path):
    """A failing rank ends the run with its status; ranks waiting on it are terminated."""
    probe = tmp_path / "probe.py"
    probe.write_text("import os, sys, time\n"
                     "if os.environ['RANK'] == '1':\n    sys.exit(7)\n"
                     "time.sleep(60)\n")
    rc = bench.spawn_ranks(3, [], poll_s=0.05, script=str(probe))
    assert rc == 7


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 2
    assert "WORLD_SIZE=1 but --gpus 2" in p.stderr


def test_bench_tools_refuse_multi_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--train", "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 2


def _record(tmp_path, sha):
    rec = {"envs": 4096, "substeps": 5, "hbm_bytes_per_launch": 2.2e7, "valu_insts_per_launch": 2.5e7}
    if sha is not None:
        rec["lib_sha256"] = sha
    path = tmp_path / "pmc.json"
    path.write_text(json.dumps(rec))
    return str(path)


def test_load_pmc_requires_the_measured_library(tmp_path):
    lib = tmp_path / "libswarmstep.so"
    lib.write_bytes(b"kernel build A")
    sha_a = bench.lib_sha256(str(lib))
    d, why = bench.load_pmc(4096, 5, str(lib), _record(tmp_path, sha_a))
    assert why is None and d["valu_insts_per_launch"] == 2.5e7
    # a rebuilt library: the record is dropped, with the reason
    lib.write_bytes(b"kernel build B")
    d, why = bench.load_pmc(4096, 5, str(lib), _record(tmp_path, sha_a))
    assert d == {} and "sha256" in why
    # an unstamped record, or one of another workload, never feeds the line
    d, why = bench.load_pmc(4096, 5, str(lib), _record(tmp_path, None))
    assert d == {} and "stamp" in why
    d, why = bench.load_pmc(8192, 5, str(lib), _record(tmp_path, bench.lib_sha256(str(lib))))
    assert d == {} and "envs=4096" in why
    # a record of the one-launch decision never feeds a 2-group line (per-decision figures differ)
    d, why = bench.load_pmc(4096, 5, str(lib), _record(tmp_path, bench.lib_sha256(str(lib))), groups=2)
    assert d == {} and "groups=1" in why


def test_roofline_per_decision_with_groups():
    """With groups, the record's per-decision figures (per-launch x groups) feed the line."""
    pmc = {"groups": 2, "valu_insts_per_launch": 1.25e7, "valu_insts_per_decision": 2.5e7,
           "hbm_bytes_per_decision": 2.2e7}
    r = bench.valu_roofline(pmc, None, 50e-6, 1000.0, 2.2e7, 4096, 5, 5.28e7, "ab", 203, 2)
    assert r["valu_insts_per_decision"] == 2.5e7 and r["groups"] == 2 and r["layout"] == 203
    assert r["frac"] == pytest.approx(2.5e7 * 64 / 50e-6 / bench.VALU_PEAK_LANE_OPS)


def test_roofline_line_shape():
    pmc = {"valu_insts_per_launch": 2.5e7, "hbm_bytes_per_launch": 2.2e7, "valu_busy": 0.5,
           "sq_wait_any_frac": 0.3}
    r = bench.valu_roofline(pmc, None, 50e-6, 1000.0, 2.2e7, 4096, 5, 5.28e7, "ab")
    assert r["bound"] == "valu" and r["unit"] == "T lane-ops/s"
    assert r["frac"] == pytest.approx(2.5e7 * 64 / 50e-6 / bench.VALU_PEAK_LANE_OPS)
    assert r["secondary"]["bound"] == "hbm" and r["secondary"]["frac"] == pytest.approx(1000.0 / 8000.0)
    r = bench.valu_roofline({}, "stale", 50e-6, 1000.0, None, 4096, 5, 5.28e7, "ab")
    assert r["achieved"] is None and r["frac"] is None and r["pmc_status"] == "stale"
