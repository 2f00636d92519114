"""bench.py's self-launch path (`python bench.py --gpus N`, N > 1, no torchrun):
the parent builds the torch.distributed.run command, never touches the GPU, and
forwards rank 0's JSON line with its CPU baseline merged in.  CPU only."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_child_command_runs_n_ranks_of_this_script():
    cmd = bench.child_command(["--gpus", "4", "--steps", "5", "--no-cpu-baseline"], 4, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    script = cmd.index(os.path.join(ROOT, "bench.py"))
    rest = cmd[script + 1:]
    assert rest[:4] == ["--gpus", "4", "--steps", "5"]
    assert rest.count("--no-cpu-baseline") == 1  # the parent ran the host legs


def test_merge_child_line_takes_rank0_json_and_adds_cpu_baseline():
    child = {"metric": "m", "value": 1.0, "n_gpus": 2, "host_legs_s": {"pmc_passes_s": 0.0},
             "xgmi": {"collective": "all_reduce"}, "cpu_baseline": None}
    out = "gloo banner\n[W something]\n" + json.dumps(child) + "\ntrailing\n"
    cpu = {"value": 5.0, "unit": "GB/s", "cores": 16, "kind": "port", "sample": "s"}
    line = bench.merge_child_line(out, cpu, {"cpu_baseline_s": 12.0}, ["py", "-m", "torch.distributed.run",
                                                                      "--nnodes=1", "--nproc-per-node=2", "a", "b"])
    assert line["n_gpus"] == 2 and line["xgmi"] == child["xgmi"]
    assert line["cpu_baseline"] == cpu
    assert line["host_legs_s"] == {"pmc_passes_s": 0.0, "parent_cpu_baseline_s": 12.0}
    assert "self-launched" in line["launch"]
    assert bench.merge_child_line("no json here\n{not json}\n", cpu, {}, ["x"] * 8) is None


def test_main_self_launches_without_torchrun_env(monkeypatch):
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    seen = {}

    def fake(args, argv):
        seen["gpus"], seen["argv"] = args.gpus, argv
        return 0

    monkeypatch.setattr(bench, "self_launch", fake)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    assert seen == {"gpus": 2, "argv": ["--gpus", "2", "--steps", "3"]}


def test_self_launch_forwards_the_child_line(monkeypatch, capsys):
    """self_launch with the child replaced by a stub that prints a rank-0 line:
    one JSON line on stdout, CPU baseline merged, child's exit code returned."""
    import subprocess
    import types
    calls = {}

    def fake_run(cmd, env=None, stdout=None, text=None):
        calls["cmd"], calls["env"] = cmd, env
        return types.SimpleNamespace(returncode=0, stdout=json.dumps({"metric": "m", "n_gpus": 2}) + "\n")

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(bench, "cpu_baseline_diloco", lambda model, K: {"value": 1.0, "cores": 2})
    args = bench.argparse.Namespace(gpus=2, no_cpu_baseline=False, only=None, model="gpt2-124m", nodes=8, replicas=None)
    assert bench.self_launch(args, ["--gpus", "2"]) == 0
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 1
    line = json.loads(out[0])
    assert line["n_gpus"] == 2 and line["cpu_baseline"] == {"value": 1.0, "cores": 2}
    assert "--nproc-per-node=2" in calls["cmd"]
    assert calls["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


@pytest.mark.parametrize("world,per_gpu", [(1, 8), (2, 4), (4, 2), (8, 1)])
def test_headline_is_eight_nodes_in_total(world, per_gpu):
    """configs[2] is 8 nodes in total: 8/N per GPU, so the driver's 1->8 curve
    runs one configuration (at N = 8 one node per GPU, the exchange over xGMI)."""
    k = bench.replicas_per_gpu(8, world)
    assert k == per_gpu and k * world == 8
    assert bench.replicas_per_gpu(8, world, override=8) == 8  # the weak-scaled extra
    with pytest.raises(SystemExit):
        bench.replicas_per_gpu(8, 3)


def test_launch_world_prefers_torchrun_env(monkeypatch):
    args = bench.argparse.Namespace(gpus=1)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.launch_world(args) == 1
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.launch_world(args) == 4
