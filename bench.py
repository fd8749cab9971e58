#!/usr/bin/env python3
"""Headline benchmark: clips/s fwd+bwd of the deformable DVC proposal path
(BaseEncoder + 6 enc + 6 dec deformable transformer + heads, T=1024, d=512, L=4 levels,
100 queries) — BASELINE.json ``metric`` / ``configs[1]`` — on N MI355X, one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W]     (N > 1: spawns the N ranks itself)
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one training iteration over one synthetic batch per GPU (8 clips): bf16 autocast
forward, backward, gradient all-reduce over RCCL (N > 1, one flat fp32 buffer),
clip_grad_norm_(0.1) and AdamW (reference engine.py:86-134, main.py:98), replayed as two
HIP graphs around the all-reduce (train_step.py; --graph 0 runs it eagerly).  Inputs are
resident in HBM before timing.
Prints ONE JSON line on rank 0, including
  roofline     — the dominant MSDA launch's algorithmic bytes / its average duration, timed
                 with HIP events on the launch stream around every MSDA C-ABI call of
                 --timer-steps eager steps run right after the timed graph replays;
  cpu_baseline — the reference's pure-PyTorch CPU path (oracle: per-level grid_sample core
                 + the same stock-PyTorch layers, fp32) timed on this host, rank 0, N=1.
"""
import argparse
import importlib
import json
import os
import platform
import subprocess
import sys
import time

# before torch touches HIP: see multimodal-feature-learning_amd/__init__.py (graph packet capture)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import torch  # noqa: E402
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = importlib.import_module("multimodal-feature-learning_amd")

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
GATHER_CEIL_TBPS = 18.8  # L2-resident indexed-row gather, chip-wide (same guide, "Indexed rows")


WORKLOADS = {
    "video": "configs[1]: models/deformable video-only, 4-level pyramid T=1024 d=512, 100 queries; "
             "BaseEncoder + 6 enc + 6 dec + heads, AdamW step",
    "multimodal": "configs[2]: multimodal video T=1024 + audio T=50 deformable fusion (4 MSDA calls per encoder "
                  "layer, 2 per decoder layer), d=512, 100 queries, 6 + 6 layers + heads, AdamW step",
    "sparse": "Sparse-DETR DVC (models/sparse, rho=0.3) T=1024 d=512, 100 queries, 6 + 6 layers, segment / count "
              "heads + mask-prediction loss through the DAM kernel, AdamW step (static top-k width: graph-captured)",
    "dvc": "full UnimodalDeformableDVC training step at configs[1] (T=1024 d=512 L=4, 100 queries, 6 + 6 layers): "
           "proposals, Hungarian matching of every decoder level, matched-segment crop, context mask, caption "
           "decoder (depth 6, vocab 10000, seq_len 20) teacher-forced on every level, criterion-shaped loss, "
           "backward, AdamW (engine.py:55-134)",
    "decode": "configs[4]'s caption AR decode at configs[1] scale: UnimodalDeformableDVC inference (T=1024 d=512 L=4, "
              "100 queries, 6 + 6 layers; proposals, matching, crops, KV-cached greedy decode of 19 words with the "
              "caption decoder depth 6, vocab 10000) on 8 clips (28 events), no_grad, bf16 autocast "
              "(engine.py:159-293 evaluate -> unimodal_deformable_dvc.py:304-354)",
}
MODELS = {"video": "DeformableDVCCore (UnimodalDeformableDVC proposal path)",
          "multimodal": "MultimodalDVCCore (MultimodalDeformableDVC proposal path)",
          "sparse": "SparseDVCCore (UnimodalSparseDVC proposal path)",
          "dvc": "UnimodalDeformableDVC (full training forward)",
          "decode": "UnimodalDeformableDVC (inference: greedy caption decode)"}


def workload_label(args):
    """configs[1] names T=1024; --T 4096 --config video is configs[3]'s per-rank shape (batch 64 over
    8 GPUs = 8 clips per rank at T=4096); other lengths are named as what they are."""
    if args.config == "video" and args.T != 1024:
        head = ("configs[3] per-rank shape: " if args.T == 4096 and args.batch == 8 else f"configs[1] at T={args.T}: ")
        return head + (f"models/deformable video-only, 4-level pyramid T={args.T} d=512, 100 queries; "
                       "BaseEncoder + 6 enc + 6 dec + heads, AdamW step")
    return WORKLOADS[args.config]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=8, help="clips per GPU")
    p.add_argument("--T", type=int, default=1024)
    p.add_argument("--queries", type=int, default=100)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    p.add_argument("--config", default="video", choices=["video", "multimodal", "sparse", "dvc", "decode"],
                   help="video: configs[1], the headline line.  multimodal: configs[2] (video + audio T_a=50, "
                        "SURVEY 8(d)); sparse: the Sparse-DETR DVC (rho=0.3; top-k width from the shapes, so it is "
                        "graph-captured too); dvc: the full UnimodalDeformableDVC training step (matching on the "
                        "host: eager), with a per-phase breakdown; decode: inference captions/s (KV-cached "
                        "greedy decode), the reference's re-decode loop timed on the CPU beside it.  Only 'video' is "
                        "the BASELINE metric's workload.")
    p.add_argument("--audio-T", type=int, default=50, help="audio length (reference audio_rescale_len)")
    p.add_argument("--dropout", type=float, default=0.1)
    p.add_argument("--cpu-baseline", type=int, default=1, help="1: time the CPU reference path (rank 0, N=1)")
    p.add_argument("--cpu-clips", type=int, default=3)
    p.add_argument("--graph", type=int, default=1, help="1: replay the step as HIP graphs (train_step.py)")
    p.add_argument("--timer-steps", type=int, default=2, help="eager steps timed per MSDA launch (roofline)")
    p.add_argument("--gemm-solutions", default=os.path.join(ROOT, "profiles", "tunableop_gfx950.csv"),
                   help="TunableOp results (hipBLASLt / rocBLAS solution per GEMM shape, tools/tune_gemms.py), "
                        "read with tuning off; 'none' = the libraries' default heuristics")
    p.add_argument("--conv-find", type=int, default=0,
                   help="1: MIOpen searches the BaseEncoder Conv1d solvers once per shape in the warm-up "
                        "(torch.backends.cudnn.benchmark; measured no gain: 712.5 vs 712.4 clips/s); 0: its immediate-mode heuristic")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                   help="per-launch HBM bytes from rocprofv3 PMC passes (profiles/), if present")
    return p.parse_args()


def cpu_model_name():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def usable_cores():
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, n)


def build_model(args, device):
    torch.manual_seed(0)
    if args.config in ("dvc", "decode"):
        return PKG.dvc_core.build_dvc(num_queries=args.queries, T=args.T, dropout=args.dropout).to(device)
    core = {"video": PKG.dvc_core.DeformableDVCCore, "multimodal": PKG.dvc_core.MultimodalDVCCore,
            "sparse": PKG.dvc_core.SparseDVCCore}[args.config]
    return core(d_model=512, num_queries=args.queries, dropout=args.dropout).to(device)


def build_batch(args, rank, device):
    if args.config in ("dvc", "decode"):
        return (PKG.dvc_core.synthetic_dvc_batch(args.batch, T=args.T, seed=1000 + rank, device=device),)
    video, mask, dur = PKG.dvc_core.synthetic_clips(args.batch, T=args.T, seed=1000 + rank, device=device)
    if args.config == "multimodal":
        audio, amask, _ = PKG.dvc_core.synthetic_clips(args.batch, T=args.audio_T, seed=2000 + rank, device=device)
        return video, mask, audio, amask, dur
    return video, mask, dur


def loss_fn(args, batch=None, model=None):
    if args.config == "dvc":
        if args.graph:  # the step around its host matching as two HIP graphs (train_step.py, staged losses)
            return PKG.dvc_core.StagedDVCLoss(batch[0], model)
        return lambda result: PKG.dvc_core.dvc_workload_loss(result, batch[0])
    return {"video": PKG.dvc_core.workload_loss, "multimodal": PKG.dvc_core.multimodal_workload_loss,
            "sparse": PKG.dvc_core.sparse_workload_loss}[args.config]


class PhaseTimer:
    """HIP events on the current stream around the full DVC step's forward phases (bench --config
    dvc): the wrapped callables record (phase, start, end); the rest of a step is backward + update."""

    def __init__(self):
        self.records, self.on = [], False

    def wrap(self, name, fn):
        def timed(*a, **kw):
            if not self.on:
                return fn(*a, **kw)
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*a, **kw)
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self.records.append((name, e0, e1))
            return r
        return timed

    def install(self, model):
        import sys as _sys
        mod = _sys.modules[type(model).__module__]
        model.forward_proposals = self.wrap("proposals_fwd", model.forward_proposals)
        model.matcher.level_costs = self.wrap("matching costs (device)", model.matcher.level_costs)
        model.matcher.solve_levels = self.wrap("matching (device->host copy, LSA on the host)",
                                               model.matcher.solve_levels)
        mod.segment_memory = self.wrap("segment crop", mod.segment_memory)
        dec = model.unimodal_caption_decoder
        dec.forward = self.wrap("caption_decoder_fwd", dec.forward)
        model.context_mask_model.forward = self.wrap("context_mask_fwd", model.context_mask_model.forward)

    def summary(self, steps, step_ms):
        tot = {}
        for name, e0, e1 in self.records:
            tot[name] = tot.get(name, 0.0) + e0.elapsed_time(e1)
        out = {k: round(v / steps, 3) for k, v in tot.items()}
        out["backward + loss + AdamW (rest of the step)"] = round(step_ms - sum(out.values()), 3)
        return out


def cpu_baseline(args):
    """The reference's CPU path: same module tree on the host, fp32, MSDA core = per-level
    F.grid_sample restatement (oracle), fwd + bwd + AdamW per clip; 1 warm-up + N timed clips."""
    from oracle.cpu_model import oracle_core
    cores = usable_cores()
    torch.set_num_threads(cores)
    torch.manual_seed(0)
    model = PKG.dvc_core.DeformableDVCCore(d_model=512, num_queries=args.queries, dropout=args.dropout)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    video, mask, dur = PKG.dvc_core.synthetic_clips(1, T=args.T, seed=0)
    times = []
    with oracle_core(PKG):
        for i in range(1 + args.cpu_clips):
            t0 = time.perf_counter()
            out = model(video, mask, dur)
            PKG.dvc_core.workload_loss(out).backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 0.1)
            opt.step()
            opt.zero_grad(set_to_none=True)
            if i:
                times.append(time.perf_counter() - t0)
    per_clip = sum(times) / len(times)
    return {"value": round(1.0 / per_clip, 4), "unit": "clips/s", "cores": cores, "kind": "port",
            "cpu": cpu_model_name(),
            "sample": f"{args.cpu_clips} clips (B=1, T={args.T}) fwd+bwd+AdamW in fp32 after 1 warm-up clip; "
                      "oracle/msda_grid_sample.py core (reference attention.py:331-383) + stock PyTorch layers"}


def decode_cpu_baseline(args):
    """The reference's inference path on this host: the same UnimodalDeformableDVC on the CPU in fp32,
    MSDA core = the per-level grid_sample restatement, captions by the reference's re-decode loop
    (oracle/cpu_model.py redecode_greedy: the whole decoder over the full prefix for every word) —
    one clip, 1 warm-up + --cpu-clips timed."""
    from oracle.cpu_model import oracle_core, reference_decode
    cores = usable_cores()
    torch.set_num_threads(cores)
    model = build_model(args, "cpu").eval()
    obj = PKG.dvc_core.synthetic_dvc_batch(1, T=args.T, seed=0)
    n_caps, times = 0, []
    with torch.no_grad(), oracle_core(PKG), reference_decode(PKG):
        for i in range(1 + args.cpu_clips):
            t0 = time.perf_counter()
            _, caps, _, _, _ = model(obj, is_training=False)
            if i:
                times.append(time.perf_counter() - t0)
                n_caps += caps.shape[0]
    return {"value": round(n_caps / sum(times), 4), "unit": "captions/s", "cores": cores, "kind": "port",
            "cpu": cpu_model_name(),
            "sample": f"{args.cpu_clips} x 1 clip (T={args.T}, {n_caps // max(1, args.cpu_clips)} events) inference in "
                      "fp32 after 1 warm-up: proposals with the oracle/msda_grid_sample.py core, the last level's "
                      "captions by the reference's full re-decode per word (unimodal_deformable_dvc.py:318-338; the "
                      "reference also re-decodes the 5 other levels every word, not charged here)"}


def run_decode(args, model, batch, world, rank):
    """--config decode: inference steps (no_grad, bf16 autocast) of UnimodalDeformableDVC; returns
    (elapsed s, captions per step, phases ms per step)."""
    model.eval()
    obj = batch[0]
    phases = PhaseTimer()
    model.forward_stage_proposals = phases.wrap("proposals + matching costs", model.forward_stage_proposals)
    dec = model.unimodal_caption_decoder
    dec.greedy_decode = phases.wrap("greedy decode (KV cache, last level)", dec.greedy_decode)

    def step():
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            return model(obj, is_training=False)[1].shape[0]

    for _ in range(args.warmup + 1):
        n_caps = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    phases.on = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    phases.on = False
    ph = phases.summary(args.steps, 1000 * elapsed / args.steps)
    ph["rest (matching on the host, crops, caption probabilities)"] = ph.pop("backward + loss + AdamW (rest of the step)")
    return elapsed, n_caps, ph


def msda_source_sha16():
    """The MSDA kernel sources' hash (as tools/pmc_summary.py records it with the PMC bytes)."""
    import hashlib
    h = hashlib.sha256()
    for f in ("msda.hip", "msda_win.hip"):
        h.update(open(os.path.join(ROOT, "multimodal-feature-learning_amd", "csrc", f), "rb").read())
    return h.hexdigest()[:16]


def roofline(summary, traffic, bursts=None, bf16=True):
    """Dominant MSDA launch kind (largest total time) -> achieved algorithmic GB/s vs HBM peak.  The
    launch duration is the burst average (KernelTimer.burst: the call re-issued back to back between
    two events) where there is one, else the single-launch event average."""
    if not summary:
        return None
    (kind, key), d = max(summary.items(), key=lambda kv: kv[1]["total_ms"])
    single = d["avg_ms"]
    d = dict(d)
    if bursts and (kind, key) in bursts:
        d["avg_ms"] = bursts[(kind, key)]
    achieved = d["bytes_per_launch"] / (d["avg_ms"] * 1e-3) / 1e9
    name = f"msda_{kind}_S{key[0]}_Lq{key[1]}"
    # (the PMC passes run the bf16 kernels: no HBM figure for an fp32 run's launch of the same shape)
    tr = traffic.get(name) if traffic and bf16 else None
    gathered = d["gather_bytes_per_launch"]
    return {"bound": "hbm", "kernel": name,
            "timing": "HIP events on the launch stream, eager steps after the timed region: around every MSDA "
                      "C-ABI call (avg_single_launch_ms, includes the ~6 us event-to-dispatch gap), and around "
                      f"{PKG.msda.KernelTimer.BURST} back-to-back re-issues of the last call of each shape "
                      "(avg_launch_ms, used for achieved). Encoder forward: msda_fwd16_tiles_kernel (also writes the "
                      "backward's tile intervals); encoder backward: win_lm_kernel (level-major row-block MFMA)",
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": tr,
            "algorithmic_bytes_per_launch": d["bytes_per_launch"], "avg_launch_ms": round(d["avg_ms"], 5),
            "avg_single_launch_ms": round(single, 5), "launches": d["launches"],
            # what actually bounds these kernels: L2/MALL-served row gathers (16 B per lane,
            # 2 taps x L*P samples per (b,q,m) item); ceiling = MI355X_MICROARCH.md "Indexed rows:
            # gather into LDS", rows resident in the XCD's L2: 16.8-18.8 TB/s chip-wide
            "gather": {"bytes_per_launch": gathered,
                       "achieved_TBps": round(gathered / (d["avg_ms"] * 1e-3) / 1e12, 2),
                       "l2_gather_ceiling_TBps": GATHER_CEIL_TBPS,
                       "frac": round(gathered / (d["avg_ms"] * 1e-3) / 1e12 / GATHER_CEIL_TBPS, 3)},
            "all_msda": {f"{k}_S{s}_Lq{q}": {"avg_ms": round(v["avg_ms"], 5), "launches": v["launches"],
                                              "burst_avg_ms": (round(bursts[(k, (s, q))], 5)
                                                               if bursts and (k, (s, q)) in bursts else None),
                                              "GBps": round(v["bytes_per_launch"] / (v["avg_ms"] * 1e-3) / 1e9, 1)}
                         for (k, (s, q)), v in summary.items()}}


def use_gemm_solutions(path):
    """Select the GEMM solutions recorded by tools/tune_gemms.py (PyTorch TunableOp over hipBLASLt
    and rocBLAS): lookups only, no tuning inside the run; shapes not in the file keep the default."""
    if not path or path == "none" or not os.path.exists(path):
        return "library default heuristics"
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(False)
    tun.record_untuned_enable(False)
    if not tun.read_file(path):
        tun.enable(False)
        return "library default heuristics (TunableOp file rejected)"
    return "TunableOp selection " + os.path.relpath(path, ROOT)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(gpus, env, argv):
    """How this invocation runs its ranks (the reference launches one DDP process per GPU,
    main.py:85 under utils/misc.py:436-458's env:// rendezvous):
      None   — run here: a launcher already started this rank (WORLD_SIZE set, equal to --gpus)
               or --gpus 1;
      [cmd]  — --gpus N > 1 and no launcher: spawn ``torch.distributed.run --nproc-per-node N``
               over 127.0.0.1 with the same arguments, as a child process (nothing here has
               touched the GPU yet), and exit with its status.
    Raises SystemExit(2) when WORLD_SIZE disagrees with --gpus: the line's n_gpus must be --gpus."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1 (got {gpus})")
    world_env = env.get("WORLD_SIZE")
    if world_env is not None:
        if int(world_env) != gpus:
            print(f"bench.py: --gpus {gpus} but WORLD_SIZE={world_env} (launcher started {world_env} ranks)",
                  file=sys.stderr, flush=True)
            raise SystemExit(2)
        return None
    if gpus == 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)


def main():
    args = parse()
    cmd = launch_plan(args.gpus, os.environ, sys.argv[1:])
    if cmd is not None:  # rank 0 of the child job prints the JSON line on the shared stdout
        sys.exit(subprocess.run(cmd).returncode)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = torch.device("cuda", local_rank)
    PKG._native.load_library()  # fail loudly before anything else if the HIP library is missing
    gemm_sel = use_gemm_solutions(args.gemm_solutions)
    torch.backends.cudnn.benchmark = bool(args.conv_find)

    model = build_model(args, device)
    if world > 1:  # identical initial weights on every rank (the reference's DDP broadcast)
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src=0)
    use_bf16 = args.dtype == "bf16"
    batch = build_batch(args, rank, device)
    if args.config == "decode":
        decode_main(args, model, batch, world, rank, device)
        return
    graph = bool(args.graph)  # dvc: two graphs around the host matching (StagedDVCLoss)
    trainer = PKG.train_step.FlatGradTrainer(model, loss_fn(args, batch, model), lr=1e-4, weight_decay=1e-4,
                                             max_norm=0.1, use_bf16=use_bf16, graph=graph)
    phases = None
    if args.config == "dvc" and not graph:
        phases = PhaseTimer()
        phases.install(model)

    trainer.capture(batch)  # eager warm-up steps + graph capture (no-op without --graph)
    for _ in range(args.warmup):
        trainer.step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if phases is not None:
        phases.on = True
    if args.config == "dvc" and graph:
        trainer.phase_events = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if phases is not None:
        phases.on = False
    graph_phases = None
    if trainer.phase_events:
        graph_phases = {}
        for name, e0, e1 in trainer.phase_events:
            dt = 1e3 * (e1 - e0) if isinstance(e0, float) else e0.elapsed_time(e1)  # (host-clock entries)
            graph_phases[name] = graph_phases.get(name, 0.0) + dt / args.steps
        graph_phases = {k: round(v, 3) for k, v in graph_phases.items()}
        trainer.phase_events = None
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # MSDA launch durations: HIP events around every C-ABI call, on the launch stream, over
    # eager steps of the same workload (events cannot bracket kernels inside a graph replay;
    # the kernels and their inputs are the same ones the graph replays)
    timer = PKG.msda.KernelTimer()
    with timer:
        for _ in range(args.timer_steps):
            trainer.eager_step(batch)
    torch.cuda.synchronize()
    summary = timer.summary()
    bursts = timer.burst() if args.timer_steps else None
    if rank == 0:
        traffic = {}
        if os.path.exists(args.traffic_json):
            try:
                traffic = json.load(open(args.traffic_json))
            except Exception:
                traffic = {}
            # PMC bytes are per kernel build: refuse them once csrc/msda.hip changed
            if traffic.get("msda_hip_sha16") != msda_source_sha16():
                traffic = {}
        clips = world * args.batch * args.steps
        result = {
            "metric": "clips/sec fwd+bwd, deformable enc/dec T=1024 d=512 L=4, 1/2/4/8 MI355X",
            "value": round(clips / elapsed, 3), "unit": "clips/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if use_bf16 else "fp32",
            "data": "synthetic (ActivityNet-shaped features N(0,1), random-init weights)",
            "config": {"workload": workload_label(args), "model": MODELS[args.config],
                       "global_batch": world * args.batch, "per_gpu_batch": args.batch, "seq_len": args.T,
                       "d_model": 512, "levels": 4, "queries": args.queries, "parallelism": f"dp{world}",
                       "execution": "hip_graph" if graph else "eager", "gemm_solutions": gemm_sel,
                       "conv_solver": "MIOpen find (cudnn.benchmark)" if args.conv_find else "MIOpen immediate"},
            "roofline": roofline(summary, traffic, bursts, bf16=use_bf16),
            "cpu_baseline": None,
        }
        if phases is not None:
            result["phases_ms_per_step"] = phases.summary(args.steps, 1000 * elapsed / args.steps)
        if graph_phases is not None:
            result["phases_ms_per_step"] = graph_phases
        if args.cpu_baseline and world == 1 and args.config == "video":
            result["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def decode_main(args, model, batch, world, rank, device):
    """bench.py --config decode: one JSON line, captions/s of the whole job (ranks decode their own
    clips: replicas, no collective), the reference's CPU re-decode beside it."""
    elapsed, n_caps, ph = run_decode(args, model, batch, world, rank)
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    timer = PKG.msda.KernelTimer()
    with timer, torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        model(batch[0], is_training=False)
    torch.cuda.synchronize()
    if rank == 0:
        caps = world * n_caps * args.steps
        result = {
            "metric": "captions/sec greedy caption decode (UnimodalDeformableDVC inference, T=1024 d=512 L=4, "
                      "100 queries), MI355X",
            "value": round(caps / elapsed, 3), "unit": "captions/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (ActivityNet-shaped features N(0,1), random-init weights)",
            "config": {"workload": WORKLOADS["decode"], "model": MODELS["decode"], "global_batch": world * args.batch,
                       "per_gpu_batch": args.batch, "captions_per_step_per_gpu": n_caps, "seq_len": args.T,
                       "caption_words": 19, "d_model": 512, "levels": 4, "queries": args.queries,
                       "parallelism": f"replicas{world}", "execution": "eager (host matching inside)"},
            "clips_per_s": round(world * args.batch * args.steps / elapsed, 3),
            "phases_ms_per_step": ph,
            "roofline": roofline(timer.summary(), {}),
            "cpu_baseline": decode_cpu_baseline(args) if args.cpu_baseline and world == 1 else None,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
