"""CPU: bench.py's own multi-rank launch (`--gpus N` without a launcher, verdict r01 #1).

spawn_ranks starts N rank processes with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT in their environment, before the parent touches torch or HIP, waits for them and exits
with the worst code; a rank that fails gets the others terminated after a grace period (a collective
would otherwise wait for it forever).  Here the ranks run a stand-in script instead of bench.py.
"""
import json
import os
import sys
import textwrap
import time

from conftest import ROOT

sys.path.insert(0, ROOT)


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_spawn_sets_the_rank_environment(tmp_path):
    import bench
    out = tmp_path / "out"
    out.mkdir()
    script = _script(tmp_path, """
        import json, os, sys
        keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"]
        json.dump({k: os.environ[k] for k in keys} | {"argv": sys.argv[1:]},
                  open(os.path.join(sys.argv[-1], os.environ["RANK"]), "w"))
    """)
    assert bench.spawn_ranks(3, ["--gpus", "3", str(out)], script=script) == 0
    got = [json.load(open(out / str(r))) for r in range(3)]
    assert [g["RANK"] for g in got] == ["0", "1", "2"] and [g["LOCAL_RANK"] for g in got] == ["0", "1", "2"]
    assert {g["WORLD_SIZE"] for g in got} == {"3"} and {g["MASTER_ADDR"] for g in got} == {"127.0.0.1"}
    assert len({g["MASTER_PORT"] for g in got}) == 1 and all(g["argv"][:2] == ["--gpus", "3"] for g in got)


def test_a_failing_rank_ends_the_others(tmp_path, monkeypatch):
    import bench
    monkeypatch.setenv("FA_BENCH_RANK_GRACE", "1")
    script = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(120)  # stands in for a rank stuck in a collective
    """)
    t0 = time.time()
    assert bench.spawn_ranks(2, [], script=script) in (3, -15)
    assert time.time() - t0 < 60
