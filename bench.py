#!/usr/bin/env python
"""Benchmark: SCFlow refinement iters/s (batch × GRU steps / s) at 256×256 on MI355X.

Workload (BASELINE.json configs[1]): a "step" is one full ``SCFlowDecoder.forward`` over a
batch of 16 synthetic 256×256 image pairs per GPU with 8 GRU refinement iterations —
correlation pyramid build, lift, and 8 × (lookup, motion encoder, SepConvGRU, heads, pose
head, pose update, reprojection, resampling) — fp32 throughout, inputs already in HBM.
Weak scaling: every rank runs its own 16 pairs (the batch shards with no collective,
SURVEY.md §8(e)); ``value`` = all pairs·iterations of all ranks ÷ the slowest rank's time.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Extra JSON fields:
* ``roofline``: the kernel with the most GPU time in the step, ``conv_wino5_kernel`` — the
  SepConvGRU's F(4,5) Winograd convolution on fp32 MFMA — over ALL four of its launches per
  refinement iteration (z|r and q of the 1×5 and the 5×1 stage), bracketed live with HIP events
  inside the timed region (each timer on one launch every other step).  ``achieved`` = Σ
  executed FLOPs of one launch of each kind ÷ Σ their mean durations; ``achieved``/``frac``
  count the FLOPs the matrix cores EXECUTE (Winograd: 8 transform points per 4-pixel tile, 5/2×
  fewer multiplies than a direct conv), so ``frac`` ≤ 1 is a true roofline fraction;
  ``direct_conv_flops_per_launch`` / ``direct_equiv_tflops`` give the direct-conv count for
  comparison.  ``traffic`` = memory-side bytes per launch from the rocprofv3 FETCH_SIZE /
  WRITE_SIZE passes in ``profiles/traffic_*.json``.
* ``rooflines_secondary``: the GRU z|r and q launches separately; the F(4×4,3×3) Winograd
  convs (XHead hidden 128→512, corr_net.1 256→192: transform launch + point-GEMM launch); the
  F(2×2,3×3) ``conv_wino_kernel<32,1>`` launches (out_net 256→126, flow_net.1 and
  delta_flow_encoder.1 128→64, mask_encoder.1 64→32); the fused lookup + corr_net.0 (or the
  pyramid lookup, HBM/gather), the pose step and the correlation pyramid — all but the GRU from
  the same events in a short untimed pass after the timed region.  HBM entries give ``frac``
  against the 8 TB/s spec and ``frac_of_measured`` against the STREAM ceiling measured on the
  box (tools/micro/stream.hip).
* ``cpu_baseline``: the CPU oracle (oracle/scflow_oracle.py, a parity-pinned PyTorch-CPU
  restatement of the reference decoder) on the same B=16 × 8-iteration workload, rank 0 at N=1.

``--gpus N`` without a launcher: the parent starts ``torch.distributed.run`` with N ranks as a
child process (before touching the GPU) and relays its output; rank 0 prints the JSON line.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "refinement iters/s (batch×GRU-steps/s) at 256×256, 1/2/4/8 MI355X"
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 = f32 vector rate


def decoder_cfg(iters, feat_size=None):
    from scflow_amd.modules import MultiClassPoseHead
    head = dict(type=MultiClassPoseHead, num_class=21, in_channels=224, net_type="Basic",
                rotation_mode="ortho6d", norm_cfg=dict(type="GN", num_groups=32, requires_grad=True),
                act_cfg=dict(type="ReLU"))
    if feat_size is not None:
        head["feat_size"] = feat_size
    # configs/refine_models/scflow_ycbv_real.py:207-230
    return dict(type="SCFlowDecoder", net_type="Basic", num_levels=4, radius=4, iters=iters,
                detach_flow=True, detach_mask=True, detach_pose=True, detach_depth_for_xy=True,
                mask_flow=False, mask_corr=False, pose_head_cfg=head,
                corr_lookup_cfg=dict(align_corners=True), gru_type="SeqConv",
                act_cfg=dict(type="ReLU"))


def make_inputs(batch, size, seed, device):
    from scflow_amd import synthetic
    raw = synthetic.make_decoder_inputs(batch, size, seed=seed)
    out = {k: torch.from_numpy(v).to(device) for k, v in raw.items()}
    out["label"] = out.pop("labels")
    return out


def encoder_cfg(norm):
    # configs/refine_models/scflow_ycbv_real.py:179-206
    return dict(type="RAFTEncoder", in_channels=3, out_channels=256, net_type="Basic",
                norm_cfg=dict(type=norm))


def build_refiner(iters, device, feat=None):
    """SCFlowRefiner (shared IN feature encoder, BN context encoder, decoder), random-init."""
    from scflow_amd import MODELS, synthetic
    r = MODELS.build(dict(type="SCFlowRefiner", cxt_channels=128, h_channels=128,
                          seperate_encoder=False, encoder=encoder_cfg("IN"),
                          cxt_encoder=encoder_cfg("BN"), decoder=decoder_cfg(iters, feat)))
    synthetic.fill_module_(r)
    return r.to(device).eval()


def make_refine_inputs(batch, size, seed, device):
    from scflow_amd import synthetic
    raw = {**synthetic.make_images(batch, size, seed=seed), **synthetic.make_scene(batch, size, seed)}
    out = {k: torch.from_numpy(v).to(device) for k, v in raw.items()}
    out["label"] = out.pop("labels")
    out.pop("init_flow", None)
    return out


def time_steps(step, steps, warmup, world, dev):
    """Warmup, then time exactly `steps` calls between barrier + synchronize; max over ranks."""
    for _ in range(warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s
# measured on the box: tools/micro/stream.hip over 2 GiB buffers (8× the Infinity Cache), best of
# 20 (profiles/r03_stream.txt): 16-B/lane read 6412 GB/s (the ceiling used here: the HBM-bound
# kernels are read-dominated), copy 4596, write 4214; the lookup's own access pattern (16-lane
# 64-B pieces in scattered order) 2803, 128-B pieces 3537.  HBM entries report frac against both.
HBM_MEASURED_GBS = 6412.0
GATHER64_MEASURED_GBS = 2803.0  # stream.hip gather_b32: the lookup's access pattern
# the 3×3 Winograd launches of one refinement iteration (decoder.kernel_hooks names): the first
# two run F(4×4,3×3) (wino4_vt_kernel + conv_wino4_kernel) by default, the rest conv_wino_kernel<32,1>
WINO_LAUNCHES = ("heads", "corr_net1", "out_net", "flow_net1", "dflow1", "mask_enc1")
# the headline kernel, conv_wino5_kernel: every SepConvGRU launch of an iteration (z|r and q of
# the 1×5 and the 5×1 stage) — the largest share of the iteration's kernel time
GRU_LAUNCHES = ("gru_zr", "gru_q")


def load_traffic(path):
    """{group: bytes per launch} from tools/traffic_json.py's output (None if absent)."""
    if not path or not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None, None
    return tj, {k: v.get("hbm_bytes_per_launch") for k, v in tj.get("kernels", {}).items()}


def conv_roofline(kernel, parts, timers, m_px, traffic=None, alg_bytes=None):
    """Roofline entry of a conv kernel symbol covering one or more launch shapes.

    ``parts`` = [(timer name, ConvRunner, c0, c1)]: achieved = Σ executed FLOPs ÷ Σ mean launch
    times, i.e. the kernel's executed rate over one launch of each shape; avg_launch_ms is the
    mean over the shapes (what rocprofv3's per-symbol average shows, one launch of each per
    iteration)."""
    ms = [timers[n].mean_ms() for n, *_ in parts]
    ex = [r.mfma_flops(m_px, c0, c1) for _, r, c0, c1 in parts]
    di = [r.flops(m_px) for _, r, _, _ in parts]
    t = sum(ms) * 1e-3
    if t <= 0:  # no timings (--no-kernel-timer: counter runs)
        return {"kernel": kernel, "bound": "mfma", "achieved": None, "peak": FP32_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s", "frac": None, "traffic": traffic}
    ach = sum(ex) / t / 1e12
    out = {"kernel": kernel, "bound": "mfma", "achieved": round(ach, 2),
           "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
           "traffic": traffic,
           "flop_basis": "executed on the matrix cores (Winograd transform-domain products, "
                         "channels padded to 32)",
           "avg_launch_ms": round(sum(ms) / len(ms), 4),
           "launches": sum(timers[n].count() for n, *_ in parts),
           "launch_ms": {n: round(v, 4) for (n, *_), v in zip(parts, ms)},
           "flops_per_launch": sum(ex) / len(ex),
           "direct_conv_flops_per_launch": sum(di) / len(di),
           "direct_equiv_tflops": round(sum(di) / t / 1e12, 2)}
    if alg_bytes is not None:
        out["algorithmic_bytes_per_launch"] = alg_bytes
        if traffic:
            out["traffic_over_algorithmic"] = round(traffic / alg_bytes, 3)
    return out


def time_fullres_alone(dec, reps=20):
    """The pose step's deferred full-resolution launch (iteration 0's recorded call) on an idle
    GPU, bracketed by the same events: its rate without the concurrent out_net / GRU launches."""
    from scflow_amd.profiling import EventTimer
    calls = getattr(dec, "_tail_calls", None)
    fc = calls[0][2] if calls else []
    if not fc:
        return None
    t = EventTimer()
    torch.cuda.synchronize()
    for _ in range(reps):
        t(True)
        for c in fc:
            c()
        t(False)
    return t.mean_ms()


def secondary_rooflines(timers, batch, size, traffic=None, fused_tail=True, tiled=True,
                        fullres_alone_ms=None):
    """The HBM/gather-bound kernels and the correlation GEMM, timed with the same events in an
    untimed pass after the timed region (algorithmic bytes per launch from SURVEY.md §8(d)).
    At B=16, 256² the 86 MB pyramid is Infinity-Cache resident, so the lookup's GB/s is an
    on-die rate; --size 512 --batch 32 --iters 12 (configs[4]) puts it in HBM."""
    h = w = size // 8
    P = h * w
    lookup_bytes = batch * (4 * P * sum(min(100, P // 4 ** l) for l in range(4)) + 4 * P * 324)
    # pose flow: 16-B point read + 8-B flow write per pixel; the fused tail (pose_step_kernel)
    # also writes the ×8 flow prediction and mask (12 B per pixel)
    flow_bytes = batch * (36 if fused_tail else 20) * size * size
    # the deferred tail's critical-path ↓8 launch: the pose flow at the 4 bilinear source pixels
    # of every feature pixel (4 × 16-B points) + the next ↓8 flow written twice (F2, HX: 16 B)
    crit_bytes = batch * P * (4 * 16 + 16)
    corr_flops = 2.0 * batch * P * P * 256
    # the lookup fused into corr_net.0 (scflow_corr_lookup_conv1x1): 2·M·324·256 flops; bytes =
    # the lookup's window reads + the 256-channel output (the 324-channel features never leave LDS)
    # + the packed weights once
    lc_flops = 2.0 * batch * P * 324 * 256
    lc_bytes = batch * (4 * P * sum(min(100, P // 4 ** l) for l in range(4)) + 4 * P * 256) + 4 * 328 * 256
    traffic = traffic or {}
    out = []
    for name, tkey, kernel, bound, amount in (
            ("corr_lookup", "corr_lookup", "corr_lookup_lds_kernel<4> (a2%s)" % (", tiled pyramid"
                                                                              if tiled else ""),
             "hbm", lookup_bytes),
            ("pose_flow", "pose_step_fullres", "pose_step_kernel (a8+a10+a11), its deferred "
             "full-resolution launch (7 per forward): queued on the side stream behind the next "
             "iteration's join, so it shares the CUs with out_net / the GRU — `achieved` is that "
             "contended rate, `alone` the same launch on an idle GPU" if fused_tail
             else "pose_flow_kernel (a8+a10)", "hbm", flow_bytes),
            ("pose_step_crit", "pose_step_crit", "pose_step_kernel (a8 + the next iteration's a11 "
             "↓8), its critical-path launch (parts = 2, 7 per forward): latency-bound, 4 "
             "workgroups per pair", "hbm", crit_bytes),
            ("corr_lookup_conv", "corr_lookup_conv", "corr_lookup_conv1x1_kernel (a2 + corr_net.0 "
             "1x1 324->256 + ReLU in one launch: the window samples go to LDS and straight into "
             "the fp32 MFMA GEMM; frac on the algorithmic flops, bytes_per_launch = window reads + "
             "output + weights)", "mfma", lc_flops),
            ("corr_pyramid", None, "corr_gemm_pyr_kernel (a1: level 0 + pooled levels 1-3 in one "
             "launch, tiled layout)" if tiled else "corr_gemm_kernel + 3 avgpool2_kernel (a1)", "mfma",
             corr_flops)):
        t = timers[name]
        if t.count() == 0:
            continue
        ms = t.mean_ms()
        if bound == "hbm":
            ach, peak, unit = amount / (ms * 1e-3) / 1e9, HBM_PEAK_GBS, "GB/s"
            extra = {"peak_measured": HBM_MEASURED_GBS,
                     "frac_of_measured": round(ach / HBM_MEASURED_GBS, 4)}
        else:
            ach, peak, unit = amount / (ms * 1e-3) / 1e12, FP32_MFMA_PEAK_TFLOPS, "TFLOP/s"
        e = {"kernel": kernel, "bound": bound, "achieved": round(ach, 2), "peak": peak,
             "unit": unit, "frac": round(ach / peak, 4), "avg_launch_ms": round(ms, 4),
             "launches": t.count(),
             ("bytes_per_launch" if bound == "hbm" else "flops_per_launch"): amount}
        if bound == "hbm":
            e.update(extra)
        if name == "corr_lookup_conv":
            e["bytes_per_launch"] = lc_bytes
            e["achieved_gbs"] = round(lc_bytes / (ms * 1e-3) / 1e9, 1)
            e["frac_of_hbm"] = round(lc_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            tr = traffic.get(tkey)
            e["traffic"] = tr
            if tr:
                e["traffic_over_algorithmic"] = round(tr / lc_bytes, 3)
        if name == "pose_flow" and fullres_alone_ms:
            e["alone"] = {"avg_launch_ms": round(fullres_alone_ms, 4),
                          "achieved": round(amount / (fullres_alone_ms * 1e-3) / 1e9, 2),
                          "frac": round(amount / (fullres_alone_ms * 1e-3) / 1e9 / peak, 4)}
        if bound == "hbm":
            tr = traffic.get(tkey)  # per launch kind (tools/traffic_json.py), or None
            e["traffic"] = tr
            if tr:
                e["traffic_over_algorithmic"] = round(tr / amount, 3)
                e["traffic_gbs"] = round(tr / (ms * 1e-3) / 1e9, 1)
            if name == "corr_lookup":  # scattered 64-B window pieces: their measured ceiling
                e["access_pattern_ceiling_gbs"] = GATHER64_MEASURED_GBS
                if tr:
                    e["traffic_frac_of_pattern_ceiling"] = round(tr / (ms * 1e-3) / 1e9 /
                                                                 GATHER64_MEASURED_GBS, 4)
        out.append(e)
    return out


def bench_train(args, world, rank, dev, feat):
    """BASELINE configs[3]: the training step — SCFlowRefiner.loss forward on the HIP kernels,
    backward through the HIP adjoint kernels, bucketed gradient all-reduce over RCCL (world > 1),
    clip 10, AdamW — `train_batch` pairs per GPU (configs[3] = 16/GPU × 8 GPUs = 128)."""
    from scflow_amd import synthetic
    from scflow_amd.train.step import TrainStep
    ref = build_refiner(args.iters, dev, feat).train()
    raw = synthetic.make_train_batch(args.train_batch, args.size, seed=2000 + rank)
    batch = {k: torch.from_numpy(v).to(dev) for k, v in raw.items()}
    pts = [torch.from_numpy(p).to(dev) for p in synthetic.make_model_points(1024)]
    step = TrainStep(ref, pts, synthetic.YCBV_DIAMETERS)
    losses = []
    evs = []
    host = []  # host seconds per step call (launching it; the step syncs only where it must)

    def one():
        # device events on the caller's stream around each step (the step orders itself after
        # and before it): the step's span on the GPU timeline, idle gaps inside it included
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        losses.append(step(batch)["loss"].detach())
        b.record()
        host.append(time.perf_counter() - t0)
        evs.append((a, b))
    # the objects the earlier legs left (decoder / refiner graphs, buffers) must not be scanned by
    # a generation-2 collection inside the timed steps: collect once, then freeze them
    gc.collect()
    gc.freeze()
    # warm up until the per-step device time is flat under the timed region's load: bursts of 6
    # back-to-back steps (a sync only at the end of a burst — per-step syncs leave the GPU idle
    # while the host refills the queue, and the clock then settles higher than under the
    # back-to-back timed steps: round 6, 18 per-step-synchronised warm-ups still drifted 37.0 →
    # 38.4 ms, profiles/r06/g10_bench.json).  Flat = the burst's last 4 steps within 1 % and its
    # median within 1 % of the previous burst's, every rank (≥ 2 and ≤ 8 bursts).
    nwarm, prev_med = 0, None
    for burst in range(8):
        for _ in range(6):
            one()
        nwarm += 6
        torch.cuda.synchronize()
        last = sorted(a.elapsed_time(b) for a, b in evs[-4:])
        med = sorted(a.elapsed_time(b) for a, b in evs[-6:])[3]
        flat = (burst >= 1 and last[-1] - last[0] <= 0.01 * last[0] and prev_med is not None and
                abs(med - prev_med) <= 0.01 * prev_med)
        prev_med = med
        if world > 1:
            f = torch.tensor([0.0 if flat else 1.0], device=dev)
            dist.all_reduce(f, op=dist.ReduceOp.MAX)
            flat = float(f.item()) == 0.0
        if flat:
            break
    el = time_steps(one, args.train_steps, 0, world, dev)
    gc.unfreeze()
    torch.cuda.synchronize()
    per_o = [a.elapsed_time(b) for a, b in evs[nwarm:]]  # the timed steps, in order
    per = sorted(per_o)
    nparam = sum(p.numel() for p in step.grads.params)
    in_sync = None
    if world > 1:  # every replica applied the same all-reduced update: parameters identical
        cs = torch.stack([p.detach().double().sum() for p in step.grads.params]).sum().reshape(1)
        allc = [torch.zeros_like(cs) for _ in range(world)]
        dist.all_gather(allc, cs)
        in_sync = all(bool(torch.equal(c, allc[0])) for c in allc)
    gb = world * args.train_batch
    which = ("BASELINE configs[3]" if (world, args.train_batch, args.size, args.iters) == (8, 16, 256, 8)
             else f"configs[3]'s per-GPU shard at N={world} (configs[3] itself is N=8, global batch 128)")
    out = {"workload": f"training step (SCFlowRefiner.loss fwd+bwd, 3 losses, grad all-reduce over "
                       f"{'RCCL' if world > 1 else 'nothing (1 rank)'}, clip, AdamW), "
                       f"{args.train_batch} pairs/GPU x {world} GPU(s) = global batch {gb}, "
                       f"{args.size}x{args.size}, {args.iters} iters — {which}",
           "value": round(gb * args.iters * args.train_steps / el, 2),
           "unit": "iters/s", "ms_per_step": round(el / args.train_steps * 1e3, 3),
           "per_step_ms": {"median": round(per[len(per) // 2], 3), "min": round(per[0], 3),
                           "max": round(per[-1], 3), "spread": round((per[-1] - per[0]) / per[len(per) // 2], 4),
                           # the first timed step starts on an idle GPU behind the barrier (its
                           # span includes the host filling the queue): spread without it too
                           "spread_after_first": round((max(per_o[1:]) - min(per_o[1:])) /
                                                       sorted(per_o[1:])[len(per_o[1:]) // 2], 4)
                           if len(per_o) > 2 else None,
                           "in_order": [round(x, 2) for x in per_o],
                           # the host's time per step call, timed steps in order: a host slower
                           # than the device shows up as device spans that follow it
                           "host_in_order": [round(1e3 * x, 2) for x in host[nwarm:]],
                           "warmup_in_order": [round(a.elapsed_time(b), 2) for a, b in evs[:nwarm]]},
           "steps": args.train_steps, "warmup": nwarm, "warmup_rule": "bursts of 6 back-to-back steps until a burst is flat (last 4 within 1 %, median within 1 % of the previous burst's)",
           "global_batch": gb, "n_gpus": world,
           "allreduce_bytes": 4 * nparam if world > 1 else 0,
           "replicas_in_sync": in_sync,
           "buckets": len(step.grads.buckets),
           "loss_first_last": [round(float(losses[0]), 4), round(float(losses[-1]), 4)]}
    del step, ref, batch
    return out


def cpu_baseline(seconds: float, batch: int, iters: int, size: int):
    """Time the CPU oracle on the bench's own workload (``batch`` pairs × ``iters`` at ``size``²),
    repeated until ``seconds`` have passed (at least one forward)."""
    from oracle import scflow_oracle as orc
    from scflow_amd import MODELS, synthetic
    feat = (size // 8, size // 8) if size != 256 else None
    dec = MODELS.build(decoder_cfg(iters, feat))
    synthetic.fill_module_(dec)
    sd = {k: v.detach() for k, v in dec.state_dict().items()}
    inp = make_inputs(batch, size, 100, "cpu")
    # torch.set_num_threads(os.cpu_count()).  On a shared box os.cpu_count()
    # counts the whole machine while this process may be confined to a share of it (affinity,
    # cgroup quota, OMP_NUM_THREADS), so the candidates are probed with one short forward each
    # and the fastest thread count runs the sample; every count is reported.
    counts = host_cpu_counts()
    cands = sorted({c for c in (counts["os_cpu_count"], counts["affinity"], counts["cgroup_quota"],
                                counts["torch_default"]) if c})
    probe = {}
    for c in cands:
        torch.set_num_threads(c)
        orc.decoder_forward(sd, **inp, iters=1)  # warm up allocator / threads
        t0 = time.perf_counter()
        orc.decoder_forward(sd, **inp, iters=1)
        probe[c] = round(time.perf_counter() - t0, 3)
    threads = min(probe, key=probe.get)
    torch.set_num_threads(threads)
    reps, t0 = 0, time.perf_counter()
    while True:
        orc.decoder_forward(sd, **inp, iters=iters)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    torch.set_num_threads(counts["torch_default"])
    return {"value": round(reps * batch * iters / el, 3), "unit": "iters/s", "cores": threads,
            "kind": "port",
            "sample": f"oracle decoder (PyTorch CPU fp32), B={batch} pairs x {iters} iters at "
                      f"{size}x{size} (the bench's own workload), {reps} forward(s) in {el:.1f}s, "
                      f"torch threads={threads} (fastest of the probed counts)",
            "host_cpus": counts, "thread_probe_s_per_1iter_forward": probe}


def host_cpu_counts():
    """os.cpu_count(), the affinity mask, the cgroup CPU quota (cpu.max) and torch's default."""
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return {"os_cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
            "cgroup_quota": quota, "torch_default": torch.get_num_threads(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def spawn_ranks(n: int) -> int:
    """`--gpus N` run directly: start torch.distributed.run with N ranks as a CHILD process (this
    process has not touched the GPU and never execs) and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd, env=dict(os.environ))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16, help="pairs per GPU")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--e2e-batch", type=int, default=32,
                    help="pairs/GPU of the extra end-to-end (images → encoders → decoder) "
                         "measurement, BASELINE configs[2]; 0 disables it")
    ap.add_argument("--e2e-steps", type=int, default=5)
    ap.add_argument("--train-batch", type=int, default=16,
                    help="pairs/GPU of the extra training-step measurement (BASELINE configs[3]); "
                         "0 disables it")
    ap.add_argument("--train-steps", type=int, default=12)
    ap.add_argument("--no-kernel-timer", action="store_true",
                    help="do not bracket the roofline kernels (throughput without timer overhead)")
    ap.add_argument("--pingpong", action="store_true",
                    help="run the batch as two interleaved halves (SCFlowDecoder.pingpong)")
    ap.add_argument("--no-tiled-pyramid", action="store_true",
                    help="row-major pyramid + separate pooling launches (SCFlowDecoder.tiled_pyramid off)")
    ap.add_argument("--graph", action="store_true",
                    help="replay a captured hipGraph per step instead of launching kernel by kernel")
    ap.add_argument("--traffic-json", default=None,
                    help="memory-side bytes per launch from rocprofv3 PMC passes "
                         "(default profiles/traffic_b{batch}_s{size}.json)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; reporting {world}",
              file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from scflow_amd import MODELS, synthetic
    from scflow_amd.modules import ConvRunner
    from scflow_amd.profiling import EventTimer, KernelTimer

    feat = (args.size // 8, args.size // 8) if args.size != 256 else None
    dec = MODELS.build(decoder_cfg(args.iters, feat))
    synthetic.fill_module_(dec)
    dec = dec.to(dev).eval()
    dec.pingpong = args.pingpong
    dec.tiled_pyramid = not args.no_tiled_pyramid
    inp = make_inputs(args.batch, args.size, seed=rank, device=dev)

    # launches per step of each bracketed kernel: 2 SeqConv stages per iteration for the z|r
    # conv, one heads / corr_net.1 / lookup / pose-flow per iteration, one pyramid per forward.
    # Eager runs bracket one launch per step per timer (stride = per-step launches + 1 walks the
    # sampled position through the iterations), so an event pair costs ≈ 2 queue packets per
    # step, not 2 per launch.
    per_step = {"gru_zr": 2 * args.iters, "gru_q": 2 * args.iters,
                "corr_lookup": args.iters, "pose_flow": args.iters,
                "pose_step_crit": args.iters, "corr_lookup_conv": args.iters, "corr_pyramid": 1}
    per_step.update({n: args.iters for n in WINO_LAUNCHES})
    # the headline kernel's launches (every conv_wino5_kernel launch of an iteration): bracketed
    # in the timed region, each timer on one launch every other step (an event pair costs a few
    # µs of queue time), the bracketed position walking through the iterations
    live = GRU_LAUNCHES
    timers = {name: (KernelTimer() if args.graph else
                     EventTimer(stride=(2 * n + 1) if name in live else (n + 1 if n > 1 else 1)))
              for name, n in per_step.items()}
    for t in timers.values():
        t.enabled = False
    if not args.no_kernel_timer:
        dec.kernel_hooks.update(timers)
    if not args.graph:
        def step():
            return dec(**inp, invalid_flow_num=0.0)
        for _ in range(args.warmup):
            step()
        for n in live:
            timers[n].enabled = True
    else:
        # one hipGraph per forward: captured after `warmup` eager passes, replayed per step
        from scflow_amd.graph import GraphedForward

        def arm():
            for t in timers.values():
                t.enabled = True
        g = GraphedForward(dec, inp, warmup=args.warmup, before_capture=arm, invalid_flow_num=0.0)
        step = g.replay

    elapsed = time_steps(step, args.steps, 0, world, dev)
    for t in timers.values():
        t.enabled = False
    if not args.graph and not args.no_kernel_timer:
        step()  # the queue refilled past the timed region's final synchronize
        for name, t in timers.items():
            t.enabled = name not in live
        for _ in range(min(args.steps, 10)):
            step()
        torch.cuda.synchronize()
        for t in timers.values():
            t.enabled = False
    fullres_alone = None if args.graph else time_fullres_alone(dec)
    dec.kernel_hooks.clear()

    e2e = None
    if args.e2e_batch > 0:
        ref = build_refiner(args.iters, dev, feat)
        rin = make_refine_inputs(args.e2e_batch, args.size, seed=1000 + rank, device=dev)
        if not args.graph:
            el2 = time_steps(lambda: ref.get_pose(**rin), args.e2e_steps, 2, world, dev)
        else:
            from scflow_amd.graph import GraphedForward
            g2 = GraphedForward(ref, rin, warmup=2, fn=ref.get_pose)
            el2 = time_steps(g2.replay, args.e2e_steps, 0, world, dev)
            del g2
        render = None
        try:  # the reference's render step in front of get_pose (format_data_test :106-117)
            from scflow_amd.renderer import Renderer
            meshes = {}
            for lab in range(21):
                semi = [a * synthetic.YCBV_DIAMETERS[lab] for a in synthetic.ELLIPSOID_AXES]
                meshes[lab] = synthetic.ellipsoid_mesh(semi, 24, 48)  # 2208 faces
            rr = Renderer(image_size=(args.size, args.size), soft_blending=False, render_mask=False,
                          seperate_lights=True, meshes=meshes).to(dev)
            rargs = (rin["ref_rotation"], rin["ref_translation"], rin["internel_k"], rin["label"])
            el3 = time_steps(lambda: rr(*rargs), args.e2e_steps, 2, world, dev)
            render = {"workload": f"HIP renderer (z-buffer + hard Phong, 2208-face meshes), "
                                  f"{args.e2e_batch} images/GPU at {args.size}x{args.size}",
                      "ms_per_batch": round(el3 / args.e2e_steps * 1e3, 3),
                      "images_per_s": round(world * args.e2e_batch * args.e2e_steps / el3, 1)}
            del rr
        except Exception as e:  # extra measurement: never take the headline down
            render = {"error": f"{type(e).__name__}: {e}"[:300]}
        e2e = {"workload": f"SCFlowRefiner.get_pose: images -> shared IN feature encoder (2 images/pair) "
                           f"+ BN context encoder + decoder, {args.e2e_batch} pairs/GPU, "
                           f"{args.size}x{args.size}, {args.iters} iters (BASELINE configs[2], "
                           f"jittered synthetic poses in place of PoseCNN init)",
               "value": round(world * args.e2e_batch * args.iters * args.e2e_steps / el2, 2),
               "unit": "iters/s", "ms_per_step": round(el2 / args.e2e_steps * 1e3, 3),
               "steps": args.e2e_steps, "warmup": 2, "render": render}
        del ref, rin

    train = None
    if args.train_batch > 0:
        try:
            train = bench_train(args, world, rank, dev, feat)
        except Exception as e:  # the extra leg must not take the headline line down with it
            train = {"error": f"{type(e).__name__}: {e}"[:400]}

    units = world * args.batch * args.iters * args.steps
    value = units / elapsed
    h8 = args.size // 8
    hb = dec.hook_batch or args.batch  # pairs per bracketed launch (a ping-pong half: batch / 2)
    m_px = hb * h8 * h8
    hc, xc = dec.h_channels, dec.cxt_channels
    tpath = args.traffic_json or os.path.join(ROOT, "profiles", f"traffic_b{hb}_s{args.size}.json")
    tj, traffic = load_traffic(tpath)
    traffic = traffic or {}
    alg = {k: v.get("algorithmic_bytes_per_launch") for k, v in (tj or {}).get("kernels", {}).items()}

    heads_r = dec._hidden_heads()

    def runner(m):
        return ConvRunner.of(m.conv, m.act_type), m.conv.in_channels
    wino = {"heads": (heads_r, hc), "corr_net1": runner(dec.encoder.corr_net[-1]),
            "out_net": runner(dec.encoder.out_net[-1]), "flow_net1": runner(dec.encoder.flow_net[-1]),
            "dflow1": runner(dec.delta_flow_encoder[-1]), "mask_enc1": runner(dec.mask_encoder[-1])}
    parts = [(n, wino[n][0], wino[n][1], 0) for n in WINO_LAUNCHES if timers[n].count()]
    cxt = xc if dec.hoist_context else 0
    zr, q = dec.gru.zr_runner(cxt), dec.gru.q_runner(cxt)
    gru = [(n, r, hc, r.cin - hc) for n, r in (("gru_zr", zr), ("gru_q", q)) if timers[n].count()]
    headline = conv_roofline(
        "conv_wino5_kernel (SepConvGRU, Winograd F(4,5) on fp32 MFMA), ALL its launches of an "
        "iteration: z|r <·,32,2,GRU_ZR> and q <·,32,1,GRU_Q> of the 1x5 and the 5x1 stage "
        "(context hoisted: K = h|r·h 128 + motion 128)",
        gru, timers, m_px, traffic.get("conv_wino5_kernel_all"), alg.get("conv_wino5_kernel_all"))
    if not all(r.winograd for _, r, _, _ in gru):
        headline["kernel"] += " [direct conv_mfma_kernel: Winograd off]"

    secondary = []
    for n, r, c0, c1 in gru:  # the two GRU launch kinds separately
        secondary.append(conv_roofline(
            {"gru_zr": "conv_wino5_kernel<·,32,2,GRU_ZR>: SepConvGRU z|r 256->256, both stages",
             "gru_q": "conv_wino5_kernel<·,32,1,GRU_Q>: SepConvGRU q 256->128, both stages"}[n],
            [(n, r, c0, c1)], timers, m_px, traffic.get(n), alg.get(n)))
    big = [p for p in parts if p[1].wino4]
    small = [p for p in parts if not p[1].wino4]
    if big:
        secondary.append(conv_roofline(
            "F(4x4,3x3) Winograd (wino4_vt_kernel input transform + conv_wino4_kernel point GEMMs "
            "and output transform; launch time = both): " +
            " + ".join({"heads": "XHead hidden 128->512" + (
                " (its launch also contracts both predictors and sums them: scflow_xhead_pred; "
                "flops counted for the hidden conv only)" if getattr(dec, "fuse_xhead_pred", False) else ""),
                "corr_net1": "corr_net.1 256->192"}.get(p[0], p[0]) for p in big),
            big, timers, m_px, traffic.get("conv_wino4"), alg.get("conv_wino4")))
    if small:
        secondary.append(conv_roofline(
            f"conv_wino_kernel<{h8},·> (F(2x2,3x3)): " + ", ".join(
                {"heads": "XHead hidden 128->512", "corr_net1": "corr_net.1 256->192",
                 "out_net": "out_net 256->126", "flow_net1": "flow_net.1 128->64",
                 "dflow1": "delta_flow_encoder.1 128->64",
                 "mask_enc1": "mask_encoder.1 64->32"}[p[0]] for p in small),
            small, timers, m_px, *((traffic.get("conv_wino_kernel<32,1>", traffic.get("conv_wino_kernel<64,*>")),
                                     alg.get("conv_wino_kernel<32,1>", alg.get("conv_wino_kernel<64,*>")))
                                    if not any(p[0] in ("heads", "corr_net1") for p in small)
                                    else (None, None))))
    secondary += secondary_rooflines(timers, hb, args.size, traffic,
                                     getattr(dec, "fuse_tail", True), dec.tiled_pyramid,
                                     fullres_alone)

    if rank == 0:
        cfg_name = ("configs[4]" if (args.batch, args.size, args.iters) == (32, 512, 12)
                    else "configs[1]" if (args.batch, args.size, args.iters) == (16, 256, 8)
                    else "custom size")
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded features, YCB-V-like poses/intrinsics, analytic ellipsoid depth; "
                    "deterministic random-init weights)",
            "config": {"workload": f"SCFlowDecoder forward, {args.batch} pairs/GPU, "
                                   f"{args.size}x{args.size}, {args.iters} GRU iters (BASELINE {cfg_name})",
                       "global_batch": args.batch * world, "image": args.size, "iters": args.iters,
                       "launch": "hipGraph replay" if args.graph else "eager",
                       "schedule": (f"two interleaved halves of {args.batch - hb} + {hb} pairs "
                                    f"(ping-pong)" if hb != args.batch else "whole batch"),
                       "parallelism": f"dp{world}"},
            "roofline": headline,
            "rooflines_secondary": secondary,
            "traffic_source": os.path.relpath(tpath, ROOT) if tj else None,
        }
        if e2e is not None:
            res["end_to_end"] = e2e
        if train is not None:
            res["training_step"] = train
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.batch, args.iters, args.size)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
