"""bench.py --gpus N without an external launcher (motionplanning_amd/launch.py): N fresh rank processes
with torch.distributed.run's environment, checked with a stub worker over gloo on CPU."""
import json
import os
import subprocess
import sys
import textwrap

from motionplanning_amd import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = textwrap.dedent("""
    import json, os, sys
    import torch, torch.distributed as dist
    out = sys.argv[1]
    env = {k: os.environ[k] for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                                      "MASTER_PORT")}
    dist.init_process_group("gloo")
    r = dist.get_rank()
    t = torch.tensor([r, int(os.environ["LOCAL_RANK"])], dtype=torch.int64)
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    with open(os.path.join(out, f"rank{r}.json"), "w") as f:
        json.dump({"env": env, "world": dist.get_world_size(), "joined": [p.tolist() for p in parts]}, f)
    dist.destroy_process_group()
""")


def test_spawn_local_two_ranks_gloo(tmp_path):
    stub = tmp_path / "stub.py"
    stub.write_text(STUB)
    st = launch.spawn_local(2, [sys.executable, str(stub), str(tmp_path)], timeout=120)
    assert st == 0
    port = None
    for r in range(2):
        d = json.loads((tmp_path / f"rank{r}.json").read_text())
        assert d["world"] == 2
        assert d["joined"] == [[0, 0], [1, 1]]
        e = d["env"]
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "2"
        assert e["MASTER_ADDR"] == "127.0.0.1"
        port = port or e["MASTER_PORT"]
        assert e["MASTER_PORT"] == port


def test_failing_rank_fails_the_job(tmp_path):
    stub = tmp_path / "bad.py"
    stub.write_text("import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(3)\ntime.sleep(60)\n")
    assert launch.spawn_local(2, [sys.executable, str(stub)], timeout=120) == 3


def test_relaunch_only_without_world_size(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert launch.relaunch_if_needed(2) is None  # already a rank (torch.distributed.run)
    monkeypatch.delenv("WORLD_SIZE")
    assert launch.relaunch_if_needed(1) is None  # --gpus 1: this process is the only rank


def test_bench_gpus_flag_reaches_the_launcher():
    """bench.py calls the launcher before any GPU call (static check: no GPU here)."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    main = src[src.index("def main():"):]
    assert main.index("relaunch_if_needed(a.gpus)") < main.index("torch.cuda.set_device")
    # n_gpus counts the distinct devices the ranks joined on (a --share-device rehearsal reports 1)
    assert '"n_gpus": len({(int(r[2]), int(r[3])) for r in joined})' in src
