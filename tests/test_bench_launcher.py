"""CPU: bench.py's own multi-process path -- the self-launcher (no torchrun), per-rank input seeding, the
barrier + max-over-ranks timing and the reductions -- driven with --dry-run over gloo (world size 2), plus
the torchrun-style env path.  On the GPU node the same code runs over RCCL with the real step."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints ONE line
    return json.loads(lines[0])


def _expected_checksum(rank, batch):
    g = torch.Generator().manual_seed(1000 + rank)
    return float((torch.rand(batch, 3, 16, 16, generator=g) * 2 - 1).double().sum())


@pytest.mark.parametrize("world", [2])
def test_self_launch_dry_run(world, tmp_path):
    out_file = tmp_path / "b.json"
    rec = _run(["--gpus", str(world), "--dry-run", "--steps", "3", "--warmup", "1", "--batch", "4",
                "--out", str(out_file)])
    assert rec == json.loads(out_file.read_text())
    assert rec["n_gpus"] == world and rec["world_size"] == world and rec["dry_run"]
    assert rec["steps"] == 3 and rec["warmup"] == 1
    assert len(rec["per_rank_ms_per_step"]) == world
    # ms_per_step is the max over ranks; value = every rank's images / that time
    assert rec["ms_per_step"] == pytest.approx(max(rec["per_rank_ms_per_step"]), abs=2e-3)
    assert rec["value"] == pytest.approx(4 * world * 1000.0 / rec["ms_per_step"], rel=1e-3)
    assert rec["config"]["global_batch"] == 4 * world and rec["config"]["per_gpu_batch"] == 4
    # each rank drew its own batch (seed 1000 + rank)
    for r in range(world):
        assert rec["rank_input_checksums"][r] == pytest.approx(_expected_checksum(r, 4), abs=1e-4)
    assert rec["scaling"] == "weak" and rec["higher_is_better"] is True
    # the 8-bit code histogram of the metric record is summed over the ranks: every rank's codes
    # counted once, the bins equal the sum of the per-rank histograms
    mr = rec["metric_record"]
    assert mr["hist_sum"] == world * 4 * 3 * 16 * 16 == mr["codes"]
    from oracle import encoder as oe
    hist = sum(torch.bincount(oe.uniform_indices(torch.rand(4, 3, 16, 16, generator=torch.Generator().manual_seed(
        1000 + r)) * 2 - 1, 8).reshape(-1).clamp(0, 255), minlength=256).double() for r in range(world))
    p = hist / hist.sum()
    assert mr["code_perplexity"] == pytest.approx(float(torch.exp(-(p * torch.log(p + 1e-10)).sum())), abs=2e-3)


def test_single_rank_dry_run():
    rec = _run(["--dry-run", "--steps", "2", "--warmup", "0", "--batch", "2"])
    assert rec["n_gpus"] == 1 and rec["world_size"] == 1 and len(rec["per_rank_ms_per_step"]) == 1


def test_gpus_mismatch_with_env_is_an_error():
    e = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="29599")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=e, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stdout + r.stderr)
