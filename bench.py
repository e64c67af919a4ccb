"""Headline benchmark: Llama-3-8B bf16 pre-training throughput (tokens/s, whole job) on N MI355X.

Config (BASELINE.json): Llama-3-8B architecture (random init, synthetic token data), sequence
length 8192, micro-batch per TP degree (MBS_BY_TP), tensor parallel TP = N (<= 8) with sequence parallelism, flash
attention, fp32 master weights + fused AdamW (ZeRO-1 when DP > 1), gradient accumulation up to the
global batch.  `--parallelism dp` instead runs TP=1 x DP=N (weak scaling).  `--pp P` runs the
BASELINE's pipeline config: TP = N / P x PP = P through NxDPPModel's 1F1B schedule (P2P over RCCL
on a side stream), global batch 32 by default (the 1F1B bubble is (P-1)/(M+P-1) for M micro-batches).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Without a launcher (no WORLD_SIZE in the environment) and N > 1, bench.py starts the N rank
processes itself (child processes, before any HIP call) and waits for them.

Times exactly K optimizer steps between barrier + device synchronisation on both sides, takes
the max over ranks, rank 0 prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# library log records go to stderr: stdout carries exactly one line, the JSON result
os.environ.setdefault("NXD_LOG_STREAM", "stderr")
# TP + SP runs (N > 1): each micro-batch as two half batches on two HIP streams with their
# collectives interleaved (parallel_layers/stream_split.py; emulated TP=8 rank at 400 GB/s per rank:
# 601 -> 532 ms per step, TP=2 over its one xGMI link 4488 -> 1839; bit-identical across runs on the
# GPU kernels).  Library default is one pass; NXD_SP_STREAMS=1 restores it here.
os.environ.setdefault("NXD_SP_STREAMS", "2")
# TP = 1 (one GPU) runs the same two staggered halves without collectives: their kernels only share
# the GPU (a GEMM of one half beside the other's attention / norm / SwiGLU): 3,071 -> 3,018 ms per
# step, same loss, alternating A/B on one box (profiles/r4_tp1_halves_bench_ab.txt).
os.environ.setdefault("NXD_SP_STREAMS_NO_SP", "1")

# Micro-batch per TP degree: TP shrinks every per-rank GEMM and the attention head count, so the
# TP>1 ranks process several sequences per micro-batch to keep MFMA tiles and the attention grid
# full (global batch unchanged; 288 GB per GPU has room for it).  Full-model step of one emulated
# TP rank (tools/emulate_tp_rank.py, real TP + SP code path, no links; profiles/r3_emulate_mbs.jsonl):
# TP-8 mbs 4 / 8: 412 / 387 ms (52 / 85 GiB); TP-4 mbs 4 / 8: 733 / 696 ms (88 / 136 GiB); TP-2 mbs
# 2 / 4: 1418 / 1373 ms (117 / 159 GiB).  The SP collectives keep their total bytes and chunk count.
# TP-1 mbs 1 / 2 on one box, alternating: 3071 / 3035 ms and 3069 / 3011 ms per step, peak 187 / 225 GiB
# allocated, 190 / 228 GiB reserved of 268 GiB (profiles/r3_bench_mbs_tp1_ab.txt).
MBS_BY_TP = {1: 2, 2: 4, 4: 8, 8: 8}
# --pp: smaller micro-batches, the 1F1B bubble is (P-1)/(M+P-1) for M micro-batches
MBS_BY_TP_PP = {1: 1, 2: 2, 4: 4, 8: 4}

BASELINE_TOKENS_PER_S = None  # the reference publishes no Llama-3-8B throughput


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq", type=int, default=8192)
    ap.add_argument("--mbs", type=int, default=None,
                    help="micro-batch size (sequences); default per TP degree (MBS_BY_TP)")
    ap.add_argument("--gbs", type=int, default=None, help="global batch (sequences per optimizer step); 8 (32 with --pp)")
    ap.add_argument("--pp", type=int, default=1, help="pipeline stages (NxDPPModel 1F1B); TP = N / pp")
    ap.add_argument("--parallelism", choices=["tp", "dp"], default="tp")
    ap.add_argument("--layers", type=int, default=None, help="override #layers (NOT the headline config)")
    ap.add_argument("--no-sp", action="store_true")
    ap.add_argument("--ckpt", default=None, help="activation checkpointing: None | full | selective")
    ap.add_argument("--lr", type=float, default=1e-5, help="AdamW learning rate (tests raise it so the loss moves)")
    ap.add_argument("--cpu", action="store_true", help="force the CPU/gloo path (plumbing tests)")
    ap.add_argument("--gloo-gpu", action="store_true",
                    help="test mode: every rank on cuda:0 with gloo collectives on staged GPU tensors (multi-rank "
                         "rehearsal of the GPU code path on a one-GPU box; not a measurement)")
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


# ---- fallback ladder ------------------------------------------------------------------------
# The first multi-rank RCCL run of this tree is the driver's node run, and a hang or crash in one
# mode must not cost the whole N-GPU number.  Every rank runs as a child process of a supervisor
# that never imports torch's GPU side or touches the GPU; if a rung fails (non-zero exit, the
# child's step watchdog, or the rung's wall budget), every rank's child is killed and all ranks
# start FRESH children with the next rung's knobs:
#   1. the defaults (two staggered SP halves on two streams, RCCL channel cap 16, SP chunking);
#   2. one stream (NXD_SP_STREAMS=1: the one-pass TP + SP step);
#   3. additionally one SP chunk, RCCL's own channel choice and normal-priority comm streams.
# The JSON line records the rung that produced it and each failed rung's exit code, reason and
# stderr tail (the watchdog's stack / flight-recorder dump).
LADDER = [
    ("defaults", {}),
    ("one_stream", {"NXD_SP_STREAMS": "1", "NXD_SP_STREAMS_NO_SP": "0"}),
    ("conservative", {"NXD_SP_STREAMS": "1", "NXD_SP_STREAMS_NO_SP": "0", "NXD_SP_CHUNKS": "1",
                      "NXD_RCCL_CHANNELS": "auto", "NXD_COMM_HIGH_PRIORITY": "0"}),
]
if os.environ.get("NXD_BENCH_LADDER", "1") == "0":
    LADDER = LADDER[:1]   # no fallback: the defaults only
LADDER_BUDGET_S = float(os.environ.get("NXD_BENCH_LADDER_BUDGET_S", "570"))   # inside the driver's 600 s
LADDER_MIN_RUNG_S = float(os.environ.get("NXD_BENCH_LADDER_MIN_RUNG_S", "120"))  # kept for each later rung
_PFX = "nxd_ladder/"


def _rung_faults(k: int):
    """Test hook: NXD_BENCH_LADDER_FAULTS="1=site@r#h:hang;2=site@r#h:exit" arms NXD_FAULT_INJECT in
    rung k only."""
    for item in filter(None, os.environ.get("NXD_BENCH_LADDER_FAULTS", "").split(";")):
        rung, spec = item.split("=", 1)
        if int(rung) == k:
            return spec
    return None


def _rung_env(base, k: int, knobs):
    env = dict(base, **knobs, NXD_BENCH_CHILD="1", NXD_BENCH_RUNG=str(k))
    env.pop("NXD_FAULT_INJECT", None)
    spec = _rung_faults(k)
    if spec:
        env["NXD_FAULT_INJECT"] = spec
    elif "NXD_FAULT_INJECT" in base and not os.environ.get("NXD_BENCH_LADDER_FAULTS"):
        env["NXD_FAULT_INJECT"] = base["NXD_FAULT_INJECT"]
    return env


class _Child:
    """One rank process of a rung: started in its own session (killed as a group), stdout / stderr
    pumped by threads; JSON result lines held back, the last stderr lines kept for the record."""

    def __init__(self, argv, env, hold_json: bool):
        import collections
        import threading

        self.json_lines = []
        self.tail = collections.deque(maxlen=40)
        self.p = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, start_new_session=True)
        self.hold_json = hold_json
        self.threads = [threading.Thread(target=self._pump, args=(self.p.stdout, sys.stdout, True), daemon=True),
                        threading.Thread(target=self._pump, args=(self.p.stderr, sys.stderr, False), daemon=True)]
        for t in self.threads:
            t.start()

    def _pump(self, src, dst, is_out):
        for raw in iter(src.readline, b""):
            line = raw.decode("utf-8", "replace")
            if is_out and self.hold_json and line.startswith("{") and '"metric"' in line:
                self.json_lines.append(line.strip())
                continue
            if not is_out:
                self.tail.append(line.rstrip("\n"))
            dst.write(line)
            dst.flush()

    def poll(self):
        return self.p.poll()

    def kill(self):
        import signal

        if self.p.poll() is None:
            for sig, wait_s in ((signal.SIGTERM, 5.0), (signal.SIGKILL, 10.0)):
                try:
                    os.killpg(self.p.pid, sig)
                except (ProcessLookupError, PermissionError):
                    pass
                try:
                    self.p.wait(timeout=wait_s)
                    break
                except subprocess.TimeoutExpired:
                    continue
        self.finish()

    def finish(self):
        for t in self.threads:
            t.join(timeout=5.0)

    def tail_text(self, n_chars=1500):
        return "\n".join(self.tail)[-n_chars:]


def _per_rank_seconds(name: str, default: str, rank: int) -> float:
    """A watchdog limit: one number for every rank, or a comma list indexed by rank (the last entry
    covers the higher ranks) -- tests give the rank that hangs the shortest limit."""
    vals = [float(v) for v in os.environ.get(name, default).split(",") if v.strip()]
    return vals[min(rank, len(vals) - 1)]


def _failure_record(k: int, name: str, knobs, rc: int, why: str, t_rung: float, first_rank, tails, killed):
    """One failed rung for the JSON history.  `first_rank` is the rank whose exit (non-zero, or its
    own watchdog's 124) ended the rung -- its stderr tail is the diagnosis.  Ranks the supervisor
    killed afterwards are listed apart with their tails: they are collateral, not the cause.  With no
    first rank (the rung's wall budget ran out) every rank was killed and every tail is kept."""
    rec = {"rung": k, "name": name, "knobs": knobs, "rc": rc, "why": why, "s": round(time.monotonic() - t_rung, 1),
           "failed_rank": first_rank, "killed_by_supervisor": sorted(killed),
           "killed_tails": {str(r): tails.get(r, "") for r in sorted(killed) if r != first_rank}}
    if first_rank is not None:
        rec["stderr_tail"] = tails.get(first_rank, "")
    else:
        rec["stderr_tail"] = "\n".join(f"[rank {r}] {t}" for r, t in sorted(tails.items()))[-3000:]
    return rec


def _rung_deadline(t_start: float, k: int) -> float:
    """Wall deadline of rung k (1-based): the budget minus what the later rungs keep in reserve."""
    return t_start + LADDER_BUDGET_S - (len(LADDER) - k) * LADDER_MIN_RUNG_S


def _emit(rec_line: str, k: int, history) -> None:
    rec = json.loads(rec_line)
    rec["attempt"] = k
    rec["ladder_rung"] = LADDER[k - 1][0]
    rec["ladder_knobs"] = LADDER[k - 1][1]
    rec["ladder_failed"] = history
    print(json.dumps(rec), flush=True)


def launch_local_ranks(argv, n: int) -> int:
    """`python bench.py --gpus N` without a launcher: start N fresh rank processes (one per GPU,
    RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set) per rung of the fallback ladder.  The parent never
    imports torch or touches the GPU and never execs.  A rung fails when any rank exits non-zero or
    the rung's wall budget runs out; its ranks are then killed and the next rung starts."""
    t0 = time.monotonic()
    history = []
    rc = 1
    for k, (name, knobs) in enumerate(LADDER, 1):
        port = str(_free_port())
        base = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                    MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=port)
        kids = [_Child(argv, _rung_env(dict(base, RANK=str(r), LOCAL_RANK=str(r)), k, knobs), hold_json=(r == 0))
                for r in range(n)]
        deadline = _rung_deadline(t0, k)
        t_rung = time.monotonic()
        why, rc, first = None, 0, None
        while True:
            codes = [c.poll() for c in kids]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                first = r
                rc = c if c > 0 else 128 - c
                why = f"rank {r} exited {c}"
                break
            if codes[0] == 0:
                break
            if time.monotonic() > deadline:
                rc, why = 124, f"rung wall budget ({deadline - t_rung:.0f} s) exhausted"
                break
            time.sleep(0.2)
        if why is None:
            grace = time.monotonic() + 20.0      # rank 0 is done: the others are in their final barrier
            while any(c.poll() is None for c in kids) and time.monotonic() < grace:
                time.sleep(0.2)
        killed = [r for r, c in enumerate(kids) if c.poll() is None]   # still running: the supervisor ends them
        for c in kids:
            c.kill()
        if why is None and kids[0].json_lines:
            _emit(kids[0].json_lines[-1], k, history)
            return 0
        if why is None:
            rc, why = 1, "rank 0 exited 0 without a result line"
        if first is None and why.startswith("rank 0 exited 0"):
            first = 0
        tails = {r: c.tail_text() for r, c in enumerate(kids)}
        history.append(_failure_record(k, name, knobs, rc, why, t_rung, first, tails, killed))
        sys.stderr.write(f"[bench] ladder rung {k} ({name}) failed: {why}\n")
        sys.stderr.flush()
    return rc


def supervise_launched_rank(argv) -> int:
    """Under torch.distributed.run (the driver's N-GPU form): this process is rank RANK's supervisor.
    It starts the rank as a child per ladder rung and agrees with the other ranks' supervisors over
    the launcher's TCPStore (host-side only) on the rung's rendezvous port, on failure and on
    success.  The children rendezvous on their own port with their own store."""
    from datetime import timedelta

    from torch.distributed import TCPStore

    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    mport = int(os.environ["MASTER_PORT"])
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
    store = TCPStore(addr, mport, world_size=None if agent else world, is_master=(not agent and rank == 0),
                     timeout=timedelta(seconds=120), wait_for_workers=False)
    t0 = time.monotonic()
    history = []
    rc = 1
    for k, (name, knobs) in enumerate(LADDER, 1):
        key = f"{_PFX}r{k}/"
        if rank == 0:
            store.set(key + "port", str(_free_port()))
        port = store.get(key + "port").decode()
        env = dict(os.environ, MASTER_PORT=port)
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        child = _Child(argv, _rung_env(env, k, knobs), hold_json=(rank == 0))
        deadline = _rung_deadline(t0, k)
        t_rung = time.monotonic()
        why, rc, done_seen, order = None, 0, None, 0
        while True:
            c = child.poll()
            if c is not None and c != 0:
                if rank != 0 and store.check([_PFX + "done"]):
                    break   # rank 0 already reported this rung's result (a late teardown failure here)
                rc, why = (c if c > 0 else 128 - c), f"rank {rank} exited {c}"
                order = store.add(key + "order", 1)   # 1 = this rank failed first
                store.set(key + "fail", why)
                break
            if c == 0:
                if rank == 0:
                    break
                if store.check([_PFX + "done"]):
                    break
            if store.check([key + "fail"]):
                rc, why = 1, "peer: " + store.get(key + "fail").decode()
                break
            if rank != 0 and store.check([_PFX + "done"]):
                done_seen = done_seen or time.monotonic()
                if time.monotonic() - done_seen > 20.0:
                    break
            if time.monotonic() > deadline:
                rc, why = 124, f"rung wall budget ({deadline - t_rung:.0f} s) exhausted"
                store.set(key + "fail", f"rank {rank}: {why}")
                break
            time.sleep(0.2)
        if why is None and rank == 0 and not child.json_lines:
            rc, why = 1, "rank 0 exited 0 without a result line"
            order = store.add(key + "order", 1)
            store.set(key + "fail", why)
        killed = child.poll() is None   # this supervisor ends a still-running child: collateral
        child.kill()
        if why is None:
            if rank == 0:
                store.set(_PFX + "done", str(k))
                _emit(child.json_lines[-1], k, history)
            return 0
        store.set(key + f"end/{rank}", json.dumps({"rc": rc, "why": why, "tail": child.tail_text(),
                                                   "order": order, "killed": killed}))
        # every rank's child of this rung is dead before anyone starts the next rung
        try:
            store.wait([key + f"end/{r}" for r in range(world)], timedelta(seconds=60))
        except Exception:
            pass
        ends = {}
        for r in range(world):
            try:
                if store.check([key + f"end/{r}"]):
                    ends[r] = json.loads(store.get(key + f"end/{r}").decode())
            except Exception:
                pass
        # the rank that failed first (lowest arrival order on the store); none when the budget ran out
        failed = sorted((e["order"], r) for r, e in ends.items() if e.get("order", 0) > 0)
        first_rank = failed[0][1] if failed else None
        first = ends.get(first_rank, ends.get(rank, {}))
        history.append(_failure_record(k, name, knobs, first.get("rc", rc), first.get("why", why), t_rung, first_rank,
                                       {r: e.get("tail", "") for r, e in ends.items()},
                                       [r for r, e in ends.items() if e.get("killed")]))
        if rank == 0:
            sys.stderr.write(f"[bench] ladder rung {k} ({name}) failed: {history[-1]['why']}\n")
            sys.stderr.flush()
    return rc


def _build(a, cfg, tp, n_micro, dev, dtype):
    """Model + optimizer through the public training API, as the reference's headline script builds
    them (examples/training/llama/tp_zero1_llama_hf_pretrain/tp_zero1_llama_hf_pretrain.py:191-238):
    `neuronx_distributed_config` -> `initialize_parallel_model` -> `initialize_parallel_optimizer`
    with ZeRO-1 + fp32 master weights + fp32 gradient accumulation (the flat fused-AdamW optimizer;
    ZeRO-1 over DP).  --pp P > 1 wraps the model in NxDPPModel (1F1B over `n_micro` micro-batches,
    even layer split)."""
    import torch

    import neuronx_distributed_llama3_2_amd as nxd
    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import LlamaDecoderLayer, LlamaForCausalLM
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps
    from neuronx_distributed_llama3_2_amd.utils.training_utils import create_partition, get_param_groups_by_weight_decay

    pcfg = None
    if a.pp > 1:
        cuts = create_partition(cfg.num_hidden_layers, a.pp)
        pcfg = {"transformer_layer_cls": LlamaDecoderLayer, "num_microbatches": n_micro, "virtual_pipeline_size": 1,
                "input_names": ["input_ids", "labels"], "broadcast_and_average_loss": True,
                "auto_partition": False, "pipeline_cuts": cuts}
    nxd_config = nxd.neuronx_distributed_config(
        tensor_parallel_size=tp, pipeline_parallel_size=a.pp, pipeline_config=pcfg,
        sequence_parallel=cfg.sequence_parallel_enabled,
        optimizer_config={"zero_one_enabled": True, "grad_clipping": True, "max_grad_norm": 1.0},
        mixed_precision_config={"use_master_weights": True, "use_fp32_grad_acc": True,
                                "use_master_weights_in_ckpt": False})
    model = nxd.initialize_parallel_model(nxd_config, LlamaForCausalLM, cfg, dtype=dtype, device=dev)
    groups = get_param_groups_by_weight_decay(model, 0.01)
    opt = nxd.initialize_parallel_optimizer(nxd_config, torch.optim.AdamW, groups, lr=a.lr, betas=(0.9, 0.95), eps=1e-8)
    assert ps.get_pipeline_model_parallel_size() == a.pp
    return model, opt


def _arm_watchdog(rank: int, timeout_s: float):
    """Host-side heartbeat (kicked every micro-step): if no progress for `timeout_s` -- a hung
    collective, a rank that died -- dump every thread's stack and this rank's last collectives
    (parallel/comm.py flight recorder) to stderr and exit 124, well inside the driver's limit."""
    from neuronx_distributed_llama3_2_amd.parallel import comm
    from neuronx_distributed_llama3_2_amd.utils.resilience import StepWatchdog

    def dump():
        sys.stderr.write(f"[bench] rank {rank}: last collectives issued:\n  " + "\n  ".join(comm.flight_record(16))
                         + "\n")
        sys.stderr.flush()

    return StepWatchdog(timeout_s, on_timeout=dump, exit_on_timeout=True, exit_code=124)


def expected_initial_loss(cfg) -> float:
    """Cross-entropy of the random-init model on random tokens: the final RMSNorm leaves unit-RMS
    hidden states, so the logits are ~N(0, sigma^2 H) with sigma = initializer_range, and
    E[logsumexp] = ln V + sigma^2 H / 2 (Llama-3-8B: 11.76 + 0.82 = 12.58; BENCH_r04 loss 12.58)."""
    import math

    return math.log(cfg.vocab_size) + 0.5 * cfg.initializer_range ** 2 * cfg.hidden_size


def _check_initial_loss(loss, cfg, dev) -> float:
    """Step-0 sanity on every rank, before anything is timed: the loss is finite and within 0.5 of
    the random-init expectation; otherwise the rung fails (exit 86) instead of timing garbage."""
    import math

    import torch
    import torch.distributed as dist

    v = float(loss.item() if torch.is_tensor(loss) else loss)
    exp = expected_initial_loss(cfg)
    bad = torch.tensor([0.0 if (math.isfinite(v) and abs(v - exp) <= 0.5) else 1.0], device=dev)
    dist.all_reduce(bad, op=dist.ReduceOp.MAX)
    if bad.item() > 0:
        sys.stderr.write(f"[bench] step-0 loss check failed on some rank (this rank: {v}, expected {exp:.3f} +- 0.5)\n")
        sys.stderr.flush()
        os._exit(86)
    return v


def main(a):
    import torch
    import torch.distributed as dist

    from neuronx_distributed_llama3_2_amd.models.llama.modeling_llama import llama_config
    from neuronx_distributed_llama3_2_amd.parallel_layers import parallel_state as ps
    from neuronx_distributed_llama3_2_amd.parallel_layers import stream_split
    from neuronx_distributed_llama3_2_amd.utils.resilience import configure_collective_watchdog, fault_point
    from neuronx_distributed_llama3_2_amd.parallel_layers.random import model_parallel_manual_seed
    from neuronx_distributed_llama3_2_amd.utils.profiling import llama_num_params, mfu, model_flops_per_token

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks")
    use_cuda = torch.cuda.is_available() and not a.cpu
    if use_cuda and a.gloo_gpu:
        local_rank = 0
    if use_cuda:
        ndev = torch.cuda.device_count()
        if local_rank >= ndev:
            raise SystemExit(f"bench: LOCAL_RANK {local_rank} but only {ndev} visible GPUs")
        torch.cuda.set_device(local_rank)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if not use_cuda:
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // world))
    backend = "nccl" if use_cuda and not a.gloo_gpu else "gloo"
    from neuronx_distributed_llama3_2_amd.parallel.rccl_env import apply_rccl_env

    apply_rccl_env(world_size=world)
    # a failed / timed-out RCCL collective tears the process down (TORCH_NCCL_ASYNC_ERROR_HANDLING)
    # instead of hanging every rank; the host watchdog below catches what that does not.  The first
    # optimizer step (startup, GEMM autotuning) gets NXD_BENCH_WATCHDOG_S, every later one
    # NXD_BENCH_STEP_WATCHDOG_S, so a hang after step 1 leaves the ladder time for its next rungs.
    wd_s = _per_rank_seconds("NXD_BENCH_WATCHDOG_S", "240", rank)
    wd_step_s = _per_rank_seconds("NXD_BENCH_STEP_WATCHDOG_S", "90", rank)
    coll_timeout = configure_collective_watchdog(2 * wd_s if wd_s > 0 else 1800.0)
    dist.init_process_group(backend, rank=rank, world_size=world, timeout=coll_timeout,
                            device_id=torch.device("cuda", local_rank) if use_cuda and backend == "nccl" else None)
    watchdog = _arm_watchdog(rank, wd_s) if wd_s > 0 else None
    dev = torch.device("cuda", local_rank) if use_cuda else torch.device("cpu")
    # preflight: one all-reduce over the whole job must see every rank (RCCL on GPU)
    probe = torch.ones(1, device=dev)
    dist.all_reduce(probe)
    comm_world = int(probe.item())
    if comm_world != world:
        raise SystemExit(f"bench: {backend} all-reduce saw {comm_world} ranks, expected {world}")

    if a.gbs is None:
        a.gbs = 32 if a.pp > 1 else 8
    if a.pp > 1:
        if world % a.pp or a.parallelism != "tp":
            raise SystemExit(f"bench: --pp {a.pp} needs --parallelism tp and a GPU count divisible by it")
        tp = min(world // a.pp, 8)
    else:
        tp = min(world, 8) if a.parallelism == "tp" else 1
    if a.pp == 1:
        ps.initialize_model_parallel(tensor_model_parallel_size=tp)
        dp = ps.get_data_parallel_size()
    else:
        dp = world // (tp * a.pp)
    model_parallel_manual_seed(1234)

    over = dict(sequence_parallel_enabled=(tp > 1 and not a.no_sp), max_position_embeddings=max(8192, a.seq))
    if a.layers is not None:
        over["num_hidden_layers"] = a.layers
    if a.ckpt == "full":
        over["activation_checkpoint"] = "full"
    elif a.ckpt == "selective":
        over["selective_checkpoint_enabled"] = True
    cfg = llama_config(a.model, **over)
    if a.mbs is None:
        a.mbs = max(1, min((MBS_BY_TP_PP if a.pp > 1 else MBS_BY_TP).get(tp, 1), a.gbs // dp))
    if a.gbs % (a.mbs * dp):
        raise SystemExit(f"bench: global batch {a.gbs} not divisible by micro-batch {a.mbs} x DP {dp}")
    accum = a.gbs // (a.mbs * dp)
    model, opt = _build(a, cfg, tp, accum, dev, torch.bfloat16)
    dp = ps.get_data_parallel_size()
    nparams_local = sum(p.numel() for p in model.parameters())
    # a fresh batch for every micro-step of every step (warmup included), generated before the timed
    # region; identical across the TP ranks of one DP rank.  Random tokens cannot be memorised, so
    # at the default learning rate the reported loss stays near ln(V) and flags numerics regressions.
    # One global token stream for every layout: step k's global batch is the same gbs sequences at
    # any TP / PP / DP split (DP rank r takes its contiguous share), so runs are comparable.
    g = torch.Generator(device="cpu").manual_seed(4321)
    n_steps = a.warmup + a.steps
    stream = torch.randint(0, cfg.vocab_size, (n_steps, a.gbs, a.seq), generator=g)
    share = a.gbs // dp
    r0 = ps.get_data_parallel_rank() * share
    batches = stream[:, r0:r0 + share].reshape(n_steps * accum, a.mbs, a.seq).to(dev)
    del stream
    cursor = [0]

    def train_step():
        if a.pp > 1:
            # one 1F1B pass over all `accum` micro-batches of this DP rank, then the optimizer step
            ids = batches[cursor[0]:cursor[0] + accum].reshape(accum * a.mbs, a.seq)
            cursor[0] += accum
            loss = model.run_train(input_ids=ids, labels=ids)
            opt.step()
            opt.zero_grad()
            return loss
        tot = None
        for i in range(accum):
            opt.set_grad_sync(i == accum - 1)
            ids = batches[cursor[0]]
            cursor[0] += 1
            fault_point("bench_microstep")   # NXD_FAULT_INJECT test site (watchdog exit path)
            out = model(ids, labels=ids)
            (out.loss / accum).backward()
            tot = out.loss.detach() if tot is None else tot + out.loss.detach()
            if watchdog is not None:
                watchdog.kick()
        opt.step()
        opt.zero_grad()
        return tot / accum   # mean over the step's micro-batches (= the pipeline path's loss)

    loss0 = None
    for w in range(a.warmup):
        loss = train_step()
        if watchdog is not None:
            watchdog.kick()
            watchdog.timeout_s = max(wd_step_s, 1.0) if wd_step_s > 0 else watchdog.timeout_s
        if w == 0:
            loss0 = _check_initial_loss(loss, cfg, dev)
    if use_cuda:
        torch.cuda.synchronize()
    dist.barrier()
    ms0 = torch.cuda.memory_stats(dev) if use_cuda else {}
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = train_step()
        if watchdog is not None:
            watchdog.kick()
    if use_cuda:
        torch.cuda.synchronize()
    dist.barrier()
    ms1 = torch.cuda.memory_stats(dev) if use_cuda else {}
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    el = float(elapsed.item())
    tokens = a.gbs * a.seq * a.steps
    value = tokens / el
    if rank == 0:
        mem = torch.cuda.max_memory_allocated(dev) / 2**30 if use_cuda else 0.0
        nparams = llama_num_params(cfg)
        fpt = model_flops_per_token(nparams, cfg.num_hidden_layers, cfg.hidden_size, a.seq)
        par = f"tp{tp}" + ("_sp" if over["sequence_parallel_enabled"] else "") + \
            (f"_pp{a.pp}_1f1b" if a.pp > 1 else "") + (f"_dp{dp}_zero1" if dp > 1 else "")
        metric = "tokens/sec (whole node) Llama-3-8B TP=8 bf16 training at 1/2/4/8 MI355X"
        if a.pp > 1:
            metric = f"tokens/sec (whole node) Llama-3-8B TP={tp} x PP={a.pp} 1F1B bf16 training"
        rec = {
            "metric": metric,
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000 * el / a.steps, 2),
            "higher_is_better": True,
            "scaling": "strong" if a.parallelism == "tp" else "weak",
            "vs_baseline": (value / BASELINE_TOKENS_PER_S) if BASELINE_TOKENS_PER_S else None,
            "dtype": "bf16",
            "data": "synthetic (fresh random token ids per micro-step, random-init weights)",
            "config": {"model": a.model if a.layers is None else f"{a.model}-{a.layers}L", "global_batch": a.gbs,
                       "micro_batch": a.mbs, "seq_len": a.seq, "parallelism": par, "grad_accum": accum,
                       "optimizer": "AdamW fp32-master" + (" ZeRO-1" if dp > 1 else ""),
                       "activation_checkpoint": a.ckpt or "none"},
            "loss": round(float(loss.item() if torch.is_tensor(loss) else loss), 4),
            "loss_step0": None if loss0 is None else round(loss0, 4),
            "comm_backend": backend,
            "comm_world_size": comm_world,
            "params_per_rank": nparams_local,
            "model_params": nparams,
            "mfu": round(mfu(value, fpt, world), 4),   # vs 2.5 PFLOP/s dense bf16 per GPU
            "peak_mem_gib": round(mem, 1),
            "peak_reserved_gib": round(torch.cuda.max_memory_reserved(dev) / 2**30, 1) if use_cuda else 0.0,
            # caching-allocator events inside the timed steps (a retry = OOM -> free cache -> device sync)
            "num_alloc_retries": int(ms1.get("num_alloc_retries", 0) - ms0.get("num_alloc_retries", 0)),
            "rccl_max_channels": os.environ.get("NCCL_MAX_NCHANNELS", "rccl default"),
            "streamk_max_cus": os.environ.get("TENSILE_STREAMK_MAX_CUS", "all"),
            "sp_streams": stream_split.parts() if (over["sequence_parallel_enabled"] or stream_split.without_sp()) else 1,
            "api": "nxd.initialize_parallel_model / initialize_parallel_optimizer",
        }
        print(json.dumps(rec), flush=True)
    if watchdog is not None:
        watchdog.stop()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    args = parse()
    ladder = os.environ.get("NXD_BENCH_LADDER", "1") == "1" and os.environ.get("NXD_BENCH_CHILD") != "1"
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1 or ladder:
            sys.exit(launch_local_ranks(sys.argv[1:], args.gpus))
    elif ladder:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            raise SystemExit(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={os.environ['WORLD_SIZE']} "
                             "ranks")
        sys.exit(supervise_launched_rank(sys.argv[1:]))
    main(args)
