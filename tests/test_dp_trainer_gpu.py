"""Data parallelism through the real trainer (reference
trainer.py:117-124 prepare / :360 DDP backward / :247-274 update): two ranks
(gloo, both on the box's one GPU — the RCCL path needs one GPU per rank) each
run VideoDecoderTrainer.__call__ + update on half of a global batch, with the
HIP-graph capture on (steps 3-4 replay), vs one rank on the whole batch.

Checked (tests/dp_trainer_worker.py writes what each rank saw):
  * the init broadcast: rank 1 starts from a different local init and ends up
    with rank 0's weights;
  * step-0 local gradients: the mean over ranks == the whole-batch gradient
    (rel <= 1e-5, f32);
  * losses: the mean of the ranks' losses == the whole-batch loss every step
    (rel <= 1e-5);
  * after 5 updates (all-reduce, clip, AdamW): both ranks hold bit-identical
    weights, == the world-1 weights (rel <= 1e-5).
With graphs on, gloo reduces in update() (a gloo collective cannot be
captured, and the eager warm-up calls run the pass the graph will hold).  The
eager accumulation test below runs the all-reduce OVERLAPPED with the backward
(bucket all-reduces launched from backward progress hooks,
trainer.OverlappedAllReduce): a bucket reduced before its last gradient
landed would break the match.  A second test runs the overlapped path on a
one-rank RCCL communicator (DV_FORCE_ALLREDUCE=1) where the collectives are
captured into the HIP graph, and checks it against the plain run.  A third
accumulates two calls per update (eager, so both calls overlap their bucket
all-reduces): the second call re-averages the part the first one already
averaged, which must leave it unchanged (a SUM there grew the
gradient by world^(calls-1)).
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dp_trainer_worker.py")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return str(s.getsockname()[1])


def _run(out, world, backend="gloo", env_extra=None):
    port = _port()
    # 1 MB buckets: the small test unet (12.5 MB of gradient) spans a dozen,
    # so the overlapped all-reduce launches most of them mid-backward
    env = dict(os.environ, DV_BUCKET_MB="1", **(env_extra or {}))
    accum = env.get("DV_TEST_ACCUM", "1")
    procs = [subprocess.Popen([sys.executable, WORKER, str(out), str(world), str(r), port, backend], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(world)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace"))
    for p, lg in zip(procs, logs):
        assert p.returncode == 0, lg[-3000:]
    return [torch.load(os.path.join(out, f"w{world}_r{r}_{backend}_a{accum}.pt"), weights_only=True)
            for r in range(world)]


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


def test_two_rank_trainer_matches_one_rank(tmp_path, parity_log):
    one = _run(tmp_path, 1)[0]
    two = _run(tmp_path, 2)
    assert one["graphed"] and all(r["graphed"] for r in two), "the replayed path did not run"
    init_err = rel(two[1]["init"], two[0]["init"])
    g_err = rel((two[0]["grad0"] + two[1]["grad0"]) / 2, one["grad0"])
    l_err = max(abs((a + b) / 2 - c) / abs(c) for a, b, c in zip(two[0]["losses"], two[1]["losses"], one["losses"]))
    p_err = rel(two[0]["params"], one["params"])
    parity_log(config="2-rank gloo trainer (dim 16, 4x3x4x32x32 global, 5 steps, graphs)", init_rel=init_err,
               grad0_rel=g_err, loss_rel_max=l_err, params_rel=p_err)
    assert init_err == 0.0, "init broadcast did not give rank 1 rank 0's weights"
    assert g_err <= 1e-5, g_err
    assert l_err <= 1e-5, l_err
    assert torch.equal(two[0]["params"], two[1]["params"]), "ranks diverged after the all-reduced updates"
    assert p_err <= 1e-5, p_err


def test_overlapped_allreduce_captured_on_one_rank_rccl(tmp_path, parity_log):
    """The overlapped bucket all-reduces inside the captured training graph
    (RCCL, one rank: the sums are identities) leave the training identical to
    the run without a process group."""
    plain = _run(tmp_path, 1)[0]
    rccl = _run(tmp_path, 1, "nccl", {"DV_FORCE_ALLREDUCE": "1"})[0]
    assert rccl["graphed"] and rccl["overlapped"], "the captured call did not include the all-reduce"
    assert rccl["buckets"] >= 8, rccl["buckets"]
    p_err = rel(rccl["params"], plain["params"])
    l_err = max(abs(a - b) / abs(b) for a, b in zip(rccl["losses"], plain["losses"]))
    parity_log(config="1-rank RCCL, overlapped all-reduce captured", params_rel=p_err, loss_rel_max=l_err,
               buckets=rccl["buckets"])
    assert p_err <= 1e-5 and l_err <= 1e-5, (p_err, l_err)


def test_two_rank_gradient_accumulation_matches_one_rank(tmp_path, parity_log):
    env = {"DV_TEST_ACCUM": "2", "DV_TEST_GRAPHS": "0"}
    one = _run(tmp_path, 1, env_extra=env)[0]
    two = _run(tmp_path, 2, env_extra=env)
    p_err = rel(two[0]["params"], one["params"])
    l_err = max(abs((a + b) / 2 - c) / abs(c) for a, b, c in zip(two[0]["losses"], two[1]["losses"], one["losses"]))
    parity_log(config="2-rank gloo trainer, 2 calls per update, eager overlapped", params_rel=p_err,
               loss_rel_max=l_err)
    assert torch.equal(two[0]["params"], two[1]["params"]), "ranks diverged"
    assert l_err <= 1e-5, l_err
    assert p_err <= 1e-5, p_err


def test_rccl_captured_accumulation_matches_plain(tmp_path, parity_log):
    """Two calls per update on the one-rank RCCL communicator, graphs on: the
    second call of each update replays the captured graph into a gradient
    that already holds the first call's (averaged) buckets."""
    env = {"DV_TEST_ACCUM": "2"}
    plain = _run(tmp_path, 1, env_extra=env)[0]
    rccl = _run(tmp_path, 1, "nccl", dict(env, DV_FORCE_ALLREDUCE="1"))[0]
    assert rccl["graphed"] and rccl["overlapped"]
    p_err = rel(rccl["params"], plain["params"])
    parity_log(config="1-rank RCCL, 2 calls per update, captured overlap", params_rel=p_err)
    assert p_err <= 1e-5, p_err


def _bench(nproc, env_extra, tmp_path):
    """bench.py under torchrun on the box's one GPU (a short run: the third
    call captures the graph, the timed steps replay it)."""
    env = dict(os.environ, **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", _port(), "bench.py", "--gpus", str(nproc),
           "--steps", "2", "--warmup", "3", "--no-cpu-baseline", "--no-roofline", "--no-sampling", "--no-fp32"]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run(cmd, cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=420)
    out = p.stdout.decode(errors="replace")
    assert p.returncode == 0, out[-4000:]
    import json
    # rank 0's one JSON line; another rank's log output may share the line
    # (two processes write to one pipe), so decode from the object's start
    line = [ln for ln in out.splitlines() if '{"metric"' in ln][-1]
    return json.JSONDecoder().raw_decode(line[line.index('{"metric"'):])[0]


def test_bench_two_ranks_gloo_shared_gpu(tmp_path):
    """The bench's N-rank path end to end at the Cfg2 model (two gloo ranks on
    the one GPU): eager warm-up, capture and replay with every 3x3 wgrad on the
    deferred split-K sums.  Round 4 found the gloo warm-up flushing those sums
    at bucket boundaries while the captured pass (no capturable collective)
    flushed once: a deferred-sum table no eager call had built."""
    rec = _bench(2, {"DV_DIST_BACKEND": "gloo", "DV_SHARE_GPU": "1"}, tmp_path)
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["value"] > 0, rec


def test_bench_one_rank_rccl_overlapped_capture(tmp_path):
    """The driver's N > 1 step on one GPU: a one-rank RCCL group with the
    bucketed all-reduce forced on (DV_FORCE_ALLREDUCE), overlapped with the
    backward and captured into the HIP graph, at the Cfg2 model."""
    rec = _bench(1, {"DV_BENCH_PG": "1", "DV_FORCE_ALLREDUCE": "1"}, tmp_path)
    assert rec["n_gpus"] == 1 and rec["value"] > 0, rec
