"""Benchmark of the CBF safety-filter hot path on MI355X (BASELINE.json metric).

Default workload (cfg4): a 1024 x 1024 jittered lattice swarm (N = 1,048,576 agents), one fused
timestep (lattice-Laplacian nominal control + cull + barrier assembly + exact QP + clip + Euler)
per step, captured in hipGraphs; the cull is the lattice-window cull on one GPU and the cell list
for the sharded stripes and the random walk (--cull, lattice_cull).  value = agent-QP solves/s over the whole job (agents
whose filter ran, counted on device).

--gpus N: one rank per GPU.  Under a launcher (torchrun: RANK / WORLD_SIZE set) this process is
one rank; without one, bench.py starts the N ranks itself as child processes and relays rank 0's
line.  The lattice is split into N row stripes: by default the SAME 1M-agent
lattice at any N (strong scaling, 1024 / N rows per GPU, as BASELINE.json's metric is quoted at
N = 1M); --weak keeps --rows rows per GPU instead.  Ranks exchange ghost rows every few steps
through ONE RCCL all-to-all (neighbour rows + guard records).  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "agent-QP solves/sec (whole node) at N=1M; timesteps/sec; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FILTER_BYTES_PER_AGENT = 64    # 32 B state in (p, u0) + 16 B u out + 16 B p_new out
STEP_BYTES_PER_AGENT = 80      # + 16 B nominal control out


def _dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def progress(msg):
    """One progress line on stderr (the driver's liveness signal; under launch_ranks every rank's
    stderr is relayed with a rank prefix).  Names the pid, so a rank can be found and signalled."""
    ws, rank, _ = _dist_env()
    sys.stderr.write(f"bench.py rank {rank}/{ws} (pid {os.getpid()}): {msg}\n")
    sys.stderr.flush()


def default_rank_timeout(args):
    """Overall limit for launch_ranks: a fresh box's first `import torch` (1-2 min), communicator
    set-up and graph captures, the timed steps and their statistics / per-step-output replays
    (generously 25 ms per step at any size), and the collective timeout once more so that a rank
    blocked in a collective has raised before the parent gives up on it."""
    return 300 + 0.025 * 4 * (args.steps + args.warmup) + args.collective_timeout


def launch_ranks(n, argv, timeout_s, grace_s=30.0):
    """--gpus N without a launcher: start N copies of this script as child processes, one rank
    each (RANK = LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), relay every rank's
    stderr (and any stdout but rank 0's JSON line) to this stderr with a "[rank r]" prefix, and
    print rank 0's one JSON line.  This parent never touches the GPU.

    Failure handling: the first rank to exit non-zero is named at once; the others get grace_s
    seconds to finish or fail on their own (a peer blocked in a collective raises at the collective
    timeout or when the connection drops), then are terminated and named.  After timeout_s seconds
    overall every rank still running is terminated and named.  Any failure makes the exit status
    non-zero (124 for the overall timeout)."""
    import threading
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE))
    out = []
    lock = threading.Lock()

    def relay(r, stream, keep):
        for line in iter(stream.readline, b""):
            if keep:
                out.append(line)
                continue
            with lock:
                sys.stderr.buffer.write(f"[rank {r}] ".encode() + line)
                sys.stderr.flush()
    threads = [threading.Thread(target=relay, args=(r, p.stdout, r == 0), daemon=True) for r, p in enumerate(procs)]
    threads += [threading.Thread(target=relay, args=(r, p.stderr, False), daemon=True) for r, p in enumerate(procs)]
    for t in threads:
        t.start()

    def note(msg):
        with lock:
            sys.stderr.write(f"bench.py (launcher): {msg}\n")
            sys.stderr.flush()

    def stop_running(why):
        running = [r for r, p in enumerate(procs) if p.poll() is None]
        if running:
            note(f"terminating rank(s) {running} ({why})")
        for r in running:
            procs[r].terminate()
        for r in running:
            try:
                procs[r].wait(timeout=20)
            except subprocess.TimeoutExpired:
                procs[r].kill()
                procs[r].wait()
        return running

    t0 = time.time()
    first_fail = None
    killed, timed_out = [], False
    while any(p.poll() is None for p in procs):
        if first_fail is None:
            bad = [(r, p.returncode) for r, p in enumerate(procs) if p.poll() not in (None, 0)]
            if bad:
                first_fail = (bad[0][0], bad[0][1], time.time())
                code = bad[0][1]
                how = f"signal {-code}" if code < 0 else f"exit code {code}"
                note(f"rank {bad[0][0]} failed first ({how}); the other ranks get {grace_s:.0f} s")
        if first_fail is not None and time.time() - first_fail[2] > grace_s:
            killed = stop_running(f"rank {first_fail[0]} failed {grace_s:.0f} s ago")
            break
        if time.time() - t0 > timeout_s:
            timed_out = True
            killed = stop_running(f"overall limit of {timeout_s:.0f} s reached")
            break
        time.sleep(0.1)
    if first_fail is None:
        # every rank ended between two polls: name the failure(s) now
        bad = [(r, p.returncode) for r, p in enumerate(procs) if p.returncode != 0]
        if bad:
            first_fail = (bad[0][0], bad[0][1], time.time())
            how = f"signal {-bad[0][1]}" if bad[0][1] < 0 else f"exit code {bad[0][1]}"
            note(f"rank {bad[0][0]} failed first ({how}; ranks {[r for r, _ in bad]} ended in the same poll)")
    for t in threads:
        t.join(timeout=10)
    codes = [p.returncode for p in procs]
    if all(c == 0 for c in codes):
        sys.stdout.write(b"".join(out).decode())
        sys.stdout.flush()
        return 0
    failed = [r for r, c in enumerate(codes) if c != 0 and r not in killed]
    note(f"FAILED: rank exit codes {codes}; failed on their own: {failed}; terminated: {killed}"
         + (f"; first failure: rank {first_fail[0]}" if first_fail else "")
         + ("; overall time limit reached" if timed_out else ""))
    if timed_out:
        return 124
    return next(c for c in codes if c != 0) if first_fail is None else (first_fail[1] if first_fail[1] > 0 else 1)


def load_pmc(config):
    """This config's section of the committed PMC summary (profiles/pmc_summary.json, written by
    tools/summarize_profile.py from tools/profile.sh runs), or {}."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_summary.json")) as f:
            return json.load(f).get(config, {})
    except (OSError, ValueError, AttributeError):
        return {}


# the timed advance phase: the filter instantiation without statistics (f = 0, large window: the
# full solve queued) and the queue kernel
ADVANCE_KERNELS = ("k_lattice_filter<true, false, false>", "k_lattice_filter_hard")
# ... of the lattice-window cull
WINDOW_KERNELS = ("k_window_tile<true, false, false>", "k_lattice_filter_hard")


def load_pmc_valu(config, kernel=ADVANCE_KERNELS[0], key="valu_busy"):
    """The kernel's VALU issue fraction from the committed PMC summary (SQ_ACTIVE_INST_VALU x 4 over
    the SIMD cycles of its dispatches, tools/summarize_profile.py), if profiled.  key
    "valu_busy_2p4ghz": the clock-corrected form (issue cycles over the traced duration at the
    2.4 GHz peak clock, a lower bound; GRBM_GUI_ACTIVE reads high on short dispatches)."""
    v = load_pmc(config).get(kernel, {}).get(key)
    return None if v is None else float(v)


def load_pmc_traffic(config, kernels=ADVANCE_KERNELS):
    """HBM bytes per launch of the advance phase (sum over its kernels) for this config, if profiled."""
    d = load_pmc(config)
    vals = [d.get(k, {}).get("hbm_bytes_per_launch") for k in kernels]
    return None if any(v is None for v in vals) else float(sum(vals))


def cpu_baseline_lattice(W, H, seed, budget_s, spacing, gain, procs=None, nominal=None, cfg2=True):
    """The reference's CPU loop (oracle/refloop.py: cross_and_rescue.py:135-160 restated, with
    cvxopt's coneqp restated) on every core of this job's host share (oracle/cpu_baseline.py):
    random egos of this workload (O(N) Python cull per ego, as the reference does at this N), and
    beside it the QP-dominated cfg2 shape (N = 100) and the C restatement on the same egos."""
    from oracle import cpu_baseline
    shape = (W, H, seed, spacing, gain, nominal)
    res = cpu_baseline.run("cfg4", budget_s, procs=procs, shape=shape)
    if cfg2:
        res["qp_dominated_cfg2"] = cpu_baseline.run("qp", budget_s, procs=procs)
    res["c_restatement"] = cpu_baseline.run("cfg4_c", min(budget_s, 5.0), procs=procs, shape=shape)
    return res


def cpu_baseline_for(args, cert_sample=None):
    """The reference's CPU path on the same inputs as this config's GPU run: a
    bounded sample on rank 0's host cores, N = 1 only (oracle/ is test infrastructure, reached
    only here, after the timed region)."""
    from oracle import cpu_baseline
    b = args.cpu_budget
    if args.config in ("cfg4", "cfg4f", "cfg4r"):
        return cpu_baseline_lattice(args.width, args.rows, args.seed, b, args.spacing, args.gain, args.cpu_procs,
                                    nominal=args.nominal, cfg2=args.config != "cfg4r")
    if args.config == "cfg3":   # every pair tested on the GPU; the reference's loop culls O(N) per ego too
        return cpu_baseline_lattice(args.width, args.rows, args.seed, b, args.spacing, args.gain, args.cpu_procs,
                                    cfg2=False)
    if args.config == "cfg5":   # meet_at_center.py:118-143 per scenario (its 16 agents vs its 32 entities)
        mid = (max(1, args.warmup) + args.steps // 2) * args.mc_inner   # the middle of the timed rollout
        return cpu_baseline.run("mc", b, procs=args.cpu_procs,
                                shape=(args.mc_scenarios, args.seed, scenarios_mc_gain(), mid))
    if args.config == "cert" and cert_sample is not None:
        return cpu_baseline_cert(*cert_sample, budget_s=min(b, 8.0))
    return None


def scenarios_mc_gain():
    from cbf_amd import scenarios
    return scenarios.MC_GAIN


def full_size_check(S, args):
    """After the timed run (untimed): one more fused step of the full swarm against the separate
    cell-list filter (cbf_filter_cells with diagnostics) on the same input state -- controls
    bit-identical, and the largest row violation over the OPTIMAL QPs (the ones whose answer the
    reference defines; north star: <= 1e-7)."""
    import torch
    from cbf_amd import swarm
    pos0 = S.pos.clone()
    S.step()
    torch.cuda.synchronize()
    # the nominal control of that step: recomputed for the consensus, the step's own for cfg4r
    vel = swarm.consensus_lattice(pos0, S.W, S.H, S.gain) if S.nominal is None else S.vel.clone()
    out = swarm.filter_swarm(S.params, pos0, vel, 0, method="cells", grid=S.grid, diag=True)
    st = out["status"]
    opt = (st & 0xFF) == 1
    viol = float(out["viol"][opt].max().item()) if bool(opt.any()) else 0.0
    return {"agents": int(pos0.shape[0]), "u_bit_identical_to_cell_filter": bool(torch.equal(out["u"], S.u)),
            "status_identical": bool(torch.equal(st, S.status)), "max_row_violation_optimal": viol,
            "optimal_fraction": float(opt.float().mean().item()),
            "relaxed_fraction": float(((st & 0xFF) == 2).float().mean().item()),
            "max_relaxations": int((st >> 8).max().item())}


def safety_report(st, steps, agents=None):
    """The rollout's safety and parity record from the device statistics of the timed steps
    (include/cbf_amd.h CBF_STAT_*).  feasible_fraction = OPTIMAL solves / solves: the share whose
    output the reference defines (an exact QP minimiser; cvxopt's iterate for an infeasible QP is
    arbitrary, cbf.py:81-87).  max_violation_optimal is the north star's "max barrier violation"
    over those; the RELAXED ones violate their original rows by construction and are reported
    separately, with the rollout's minimum distance between culled neighbours."""
    n = max(st["solves"], 1)
    d2 = st["min_dist2"]
    return {"steps": steps, "solves": st["solves"],
            "feasible_fraction": st["optimal"] / n, "relaxed_fraction": st["relaxed"] / n,
            "infeasible_fraction": st["infeasible"] / n, "binding_fraction": st["binding"] / n,
            "seidel_fraction": st["seidel"] / n,
            "max_violation_optimal": st["viol_optimal"],
            "max_violation_original_rows_relaxed": st["viol_original_relaxed"],
            "min_pairwise_distance": None if d2 is None else float(np.sqrt(d2)),
            # the window cull's degradation (CBF_STAT_WIN_WALKS / GUARD_STALLS; 0 under the cell list)
            "window_walk_fraction": None if not agents else st.get("win_walks", 0) / (agents * steps),
            "window_guard_stall_words": st.get("guard_stalls", 0),
            "min_pairwise_distance_note": "over neighbour pairs the reference culls (0 < d < 0.2, "
                                          "cross_and_rescue.py:147-150); None = no pair closer than 0.2"}


def lattice_geometry(args, ws):
    """(rows per rank, whole-lattice rows, ghost-row halo, sub-steps per exchange).  Strong
    scaling (default): the --rows-row lattice split into ws stripes; --weak: --rows rows per rank.
    The halo is the rows one timestep can reach (4 for the consensus lattice; 10 for cfg4r's
    random walk, whose RELAXED QPs move an agent up to T max_speed = 0.5 per step); the sub-steps
    default to as many as fit twice into a stripe, at most 8."""
    if args.weak or ws == 1:
        R = args.rows
    else:
        if args.rows % ws:
            raise SystemExit(f"bench.py: --rows {args.rows} is not divisible into {ws} stripes (or use --weak)")
        R = args.rows // ws
    halo = 10 if args.nominal is not None else 4
    # sub-steps per exchange: a stripe of <= 512 rows does not fill the chip, so ghost rows are nearly
    # free and fewer exchanges pay (128 rows: 30.2 vs 32.3 us/step at 16 vs 8; 256: 41.8-42.2 vs 43.7;
    # 512: 57.5-57.9 vs 58.4-60.0; tools/records/gpu_r03r.sh, gpu_r03s.sh); 1024-row stripes keep 8
    cap = 16 if R <= 512 else 8
    k = args.substeps if args.substeps else max(1, min(cap, R // (2 * halo)))
    if halo * k > R:
        raise SystemExit(f"bench.py: {k} sub-steps x {halo} halo rows do not fit a stripe of {R} rows")
    return R, R * ws, halo, k


def gather_state_sha(own, ws):
    """sha256 of the whole lattice's positions (the ranks' owned rows in rank order, float64 bytes):
    the same digest for the same rollout at any rank count."""
    import torch
    x = own.contiguous()
    if ws > 1:
        import torch.distributed as dist
        if dist.get_backend() == "gloo":
            x = x.cpu()
            parts = [torch.empty_like(x) for _ in range(ws)]
            dist.all_gather(parts, x)
            x = torch.cat(parts)
        else:
            full = torch.empty((ws * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
            dist.all_gather_into_tensor(full, x)
            x = full
    return hashlib.sha256(x.cpu().numpy().tobytes()).hexdigest()


def solves_inline(cp, n):
    """Where a window of n agents solves its full QPs under the params cp actually passed
    (include/cbf_amd_measure.h cbf_lattice_solves_inline): the filter kernel, or the queue kernel."""
    from cbf_amd import _lib
    return bool(_lib.lib.cbf_lattice_solves_inline(_lib.C.byref(cp), int(n)))


def lattice_cull(args, sharded, rows=None):
    """The cull of the lattice step: --cull, or auto = the lattice-window cull (CBF_RUN_WINDOW_CULL)
    for a lattice that stays lattice-like (the consensus nominal control of cfg4 / cfg4f), the
    cell list for the random walk of cfg4r (which scrambles each row's x order: 237.7 vs 84.9 us,
    profiles/r04_cfg4r_window_vs_cells.txt) and the HOCBF barrier.  One GPU: 66.1-67.9 vs
    71.2-72.2 us per timestep at 1 M agents (profiles/r04_row_guard_ab.txt).  Sharded stripes of
    rows >= 256 rows per rank (the N <= 4 strong-scaling shares and weak scaling): one rank's
    exchange cycle 76.0 / 52.6 / 39.8 vs 87.0 / 58.1 / 42.4 us at 1024 / 512 / 256 rows; at 128
    rows (N = 8) the cell list stays, 30.4-30.6 vs 30.8-31.1 (profiles/r04_shard_window_vs_cells.txt)."""
    if args.barrier != "reference" or not 4 <= args.width <= 2048:
        if args.cull == "window":
            raise SystemExit("--cull window: reference barrier, 4 <= width <= 2048 only")
        return "cells"
    if args.cull != "auto":
        return args.cull
    if args.nominal is not None:
        return "cells"
    return "window" if not sharded or (rows is not None and rows >= 256) else "cells"


def bench_lattice(args, ws, rank, local):
    import torch
    from cbf_amd import scenarios, swarm
    W = args.width
    sharded = ws > 1 or args.shard
    rows, rows_total, halo, k = lattice_geometry(args, ws)
    if sharded:
        from cbf_amd.shard import ShardedLattice
        S = ShardedLattice(W, rows, seed=args.seed, halo=halo, substeps=k, spacing=args.spacing, gain=args.gain,
                           nominal=args.nominal, exchange=args.exchange, cull=lattice_cull(args, sharded, rows))
    else:
        pos = scenarios.lattice(W, rows, seed=args.seed, spacing=args.spacing)
        S = swarm.LatticeSwarm(pos, W, rows, gain=args.gain, barrier=args.barrier, nominal=args.nominal,
                               cull=lattice_cull(args, sharded, rows))
    progress(f"{args.config}: {W}x{rows_total} lattice built ({rows} rows on this rank)")
    use_graph = not args.eager
    # single GPU, reference barrier: the timesteps run as cbf_lattice_run calls of `chunk`
    # timesteps (bit-identical to as many cbf_lattice_step calls; each advance bins the next
    # timestep, so the bin pass runs once per call), each call one hipGraph.  Sharded: one
    # hipGraph per exchange cycle (cbf_lattice_cycle_sharded) replayed after each exchange, whose
    # pack / collective / unpack stay eager.
    # (the HOCBF barrier: `chunk` single-timestep launches captured as one graph)
    chunk = args.chunk if (use_graph and not sharded and args.chunk > 1) else 1
    plan = [chunk] * (args.steps // chunk) + ([args.steps % chunk] if args.steps % chunk else [])

    def advance(n):
        if chunk > 1 or sharded:  # sharded: whole exchange cycles as one cbf_lattice_cycle_sharded call
            S.run(n)
        else:
            for _ in range(n):
                S.step()
    # The timed rollout runs the filter path alone (stats=NULL: the reference computes no such
    # record); the safety record then comes from a replay of the same steps from the same device
    # state with the statistics on, checked bit-identical to the timed one and timed as well
    # (ms_per_step_with_stats).  --timed-stats keeps the statistics inside the timed region.
    modes = (True,) if args.timed_stats else (False, True)
    if use_graph and sharded:
        for cs in modes:   # (capture_cycle launches nothing)
            S.collect_stats = cs
            S.capture_cycle()
    elif use_graph:
        # a capture's eager warm-up launch advances the swarm: restore it afterwards, so that the
        # timed steps are timesteps W+1 .. W+K of the rollout whatever the graphs' sizes
        snap0 = S.snapshot()
        for cs in modes:
            S.collect_stats = cs
            if chunk > 1:
                for n in set(plan):
                    S.capture(steps=n)
            else:
                S.capture()
        if chunk > 1 and not args.timed_stats and args.barrier == "reference":
            # the per-step-outputs variant (history), statistics off
            S.collect_stats = False
            for n in set(plan):
                S.capture(steps=n, history=True)
        S.restore(snap0)
        del snap0
    S.collect_stats = modes[0]
    if sharded:
        # first-use costs (the collective's buffers and connections, allocations) are paid by two
        # throwaway exchange cycles, undone by restoring the state: the timed steps stay W+1 .. W+K
        snap0 = S.snapshot()
        S.run(2 * k)
        torch.cuda.synchronize()
        if ws > 1:
            S.check_guard()
        S.restore(snap0)
        del snap0
    progress(f"{args.config}: graphs captured; {args.warmup} warm-up steps")
    advance(args.warmup)
    torch.cuda.synchronize()
    snap = S.snapshot() if len(modes) > 1 else None
    S.reset_solves()
    progress(f"{args.config}: timed region ({args.steps} steps)")

    def timed(history=False):
        if ws > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if chunk > 1:
            for n in plan:
                S.run(n, history=True) if history else S.run(n)
        else:
            advance(args.steps)
        torch.cuda.synchronize()
        if ws > 1:
            torch.distributed.barrier()
        return time.perf_counter() - t0

    def max_over_ranks(x):
        if ws == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        return float(t[0])

    # the window cull's degradation counters (workspace header, counted whatever collect_stats says)
    # around the timed steps themselves: egos that walked, guard words read at their spin limit
    wc = hasattr(S, "window_counters") and S.cull == "window"
    wc0 = S.window_counters() if wc else None
    elapsed = max_over_ranks(timed())
    wc1 = S.window_counters() if wc else None
    progress(f"{args.config}: timed region done ({elapsed / args.steps * 1e6:.1f} us/step); replays")
    own = S.own if sharded else S.pos
    end_state = (own.clone(), S.u.clone(), S.status.clone())
    if ws > 1:
        S.check_guard()
    elapsed_stats = None
    if snap is not None:  # the statistics replay of the timed steps
        S.restore(snap)
        S.collect_stats = True
        S.reset_solves()
        elapsed_stats = max_over_ranks(timed())
        same = all(bool(torch.equal(a, b)) for a, b in zip(end_state, (own, S.u, S.status)))
        if ws > 1:
            f = torch.tensor([0 if same else 1], dtype=torch.int32, device="cuda")
            torch.distributed.all_reduce(f)
            same = int(f[0]) == 0
            S.check_guard()
        if not same:
            raise RuntimeError("the statistics replay did not repeat the timed rollout bit for bit")
    state_sha = gather_state_sha(own, ws)
    elapsed_hist = None
    if snap is not None and chunk > 1 and args.barrier == "reference":
        # the same timed steps again with every timestep's outputs stored (u, status, nominal
        # control, neighbour count: the reference's per-step si_velocities), statistics off
        stats_keep = S.stats.clone()
        S.restore(snap)
        S.collect_stats = False
        elapsed_hist = timed(history=True)
        if not all(bool(torch.equal(a, b)) for a, b in zip(end_state, (own, S.history(plan[-1])[1][-1],
                                                                       S.history(plan[-1])[2][-1]))):
            raise RuntimeError("the per-step-outputs run did not repeat the timed rollout bit for bit")
        S.stats.copy_(stats_keep)
        S.collect_stats = True
    if snap is not None:
        del snap
    solves = S.solves_total()
    n_local = S.n_owned if sharded else S.n
    if ws > 1:
        t = torch.tensor([float(solves), float(n_local)], dtype=torch.float64, device="cuda")
        torch.distributed.all_reduce(t)
        solves = int(t[0]); n_total = int(t[1])
    else:
        n_total = n_local
    # the timed rollout's safety record, before the kernel-timing launches below add to it
    stat = S.stats_summary()
    if ws > 1:
        import torch.distributed as dist
        keys = ("solves", "optimal", "relaxed", "infeasible", "seidel", "binding")
        c = torch.tensor([stat[k] for k in keys], dtype=torch.float64, device="cuda")
        m = torch.tensor([stat["viol_optimal"], stat["viol_original_relaxed"],
                          -(stat["min_dist2"] if stat["min_dist2"] is not None else np.inf)],
                         dtype=torch.float64, device="cuda")
        dist.all_reduce(c)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        stat.update({k: int(v) for k, v in zip(keys, c.tolist())})
        stat.update(viol_optimal=float(m[0]), viol_original_relaxed=float(m[1]),
                    min_dist2=None if not np.isfinite(m[2].item()) else -float(m[2]))
    safety = safety_report(stat, args.steps, n_total) if args.barrier == "reference" else None
    window_cull = None
    if wc:
        window_cull = {"walk_fraction": (wc1[0] - wc0[0]) / (n_local * args.steps),
                       "guard_stall_words": wc1[1] - wc0[1],
                       "note": "over the timed steps: egos per timestep that took the unbounded row walk, and "
                               "row-guard words read at their spin limit (cbf_lattice_window_counters); both "
                               "stay exact, both say the swarm has left the window cull's fast path"}
    exchange = None
    if sharded:
        # each rank's exchange (pack + collective + unpack with the guard), timed alone after the
        # rollout, gathered to rank 0: the per-rank cost the strong-scaled step pays per timestep
        ex = S.time_exchange(10)
        keys = ("pack_us", "collective_us", "unpack_guard_us", "exchange_us", "exchange_us_per_timestep")
        mine = torch.tensor([ex[k] for k in keys], dtype=torch.float64, device="cuda")
        rows_all = [mine]
        if ws > 1:
            rows_all = [torch.empty_like(mine) for _ in range(ws)]
            torch.distributed.all_gather(rows_all, mine)
        per_rank = [dict(zip(keys, (float(v) for v in r.tolist()))) for r in rows_all]
        exchange = {"per_rank": per_rank,
                    "max_exchange_us_per_timestep": max(r["exchange_us_per_timestep"] for r in per_rank),
                    "timesteps_per_exchange": k, "bytes_sent_per_rank": S.exchange_bytes(),
                    "note": "pack + collective + unpack/guard, each closed by a device synchronize, mean of 10 "
                            "exchanges timed after the rollout (state restored); the timed steps overlap none of "
                            "it with compute, so it is part of ms_per_step"}
    comm = ("RCCL" if args.backend == "nccl" else "gloo (host-staged rehearsal)") if ws > 1 else "single-rank"
    # dominant kernel (filter + clip + Euler) timed alone with HIP events on the launch stream
    S.collect_stats = modes[0]  # as in the timed region
    # the dominant kernel (k_lattice_filter) alone: an event recorded by the advance call between
    # it and the queued-QP kernel, on their launch stream (reference barrier)
    marked = args.barrier == "reference"
    cull = getattr(S, "cull", None) or getattr(getattr(S, "be", None), "cull", "cells")
    kt = []
    # the GPU is kept busy (a spin kernel) while the host enqueues the start event and the advance,
    # so the events time the kernels and not the host's launch latency (a 20-us window-cull build
    # can drain before the host has launched the advance)
    spin = getattr(torch.cuda, "_sleep", None)
    # single GPU: the filter is also launched with hipExtLaunchKernel start / stop events, which
    # carry the dispatch's own start and end (as a kernel trace measures it); the stream events
    # around it also cover the dispatch of the launch and its end-of-kernel cache flush
    own = marked and not sharded
    kt, ko = [], []
    for it in range(args.kernel_iters * (2 if own else 1)):
        timed_launch = own and it % 2 == 1
        S.build_phase()
        a, m, b, fs, fe = (torch.cuda.Event(enable_timing=True) for _ in range(5))
        if marked:
            m.record()   # creates the event; the advance call records it again after the filter
        if timed_launch:
            fs.record()  # created here; the filter's launch sets both
            fe.record()
        if spin is not None:
            spin(200000)
        a.record()
        if timed_launch:
            S.advance_phase(timing=(fs, fe), **({"commit": False} if cull == "window" else {}))
        elif marked and cull == "window":
            S.advance_phase(mark=m, commit=False)   # (the new positions into scratch: no copy timed)
        elif marked:
            S.advance_phase(mark=m)
        else:
            S.advance_phase()
        b.record()
        (ko if timed_launch else kt).append((a, m, b, fs, fe))
    torch.cuda.synchronize()
    k_ms = float(np.mean([a.elapsed_time(b) for a, m, b, fs, fe in kt]))
    f_stream_ms = float(np.mean([a.elapsed_time(m) for a, m, b, fs, fe in kt])) if marked else k_ms
    f_ms = float(np.mean([fs.elapsed_time(fe) for a, m, b, fs, fe in ko])) if own else f_stream_ms
    status = S.status.cpu().numpy()
    codes = np.bincount(status & 0xFF, minlength=5)
    check = full_size_check(S, args) if (ws == 1 and not args.shard and args.barrier == "reference") else None
    achieved = FILTER_BYTES_PER_AGENT * n_local / (f_ms * 1e-3) / 1e9
    achieved_adv = FILTER_BYTES_PER_AGENT * n_local / (k_ms * 1e-3) / 1e9
    adv_kernels = WINDOW_KERNELS if cull == "window" else ADVANCE_KERNELS
    traffic = load_pmc_traffic(args.config, adv_kernels[:1]) if args.barrier == "reference" else \
        load_pmc_traffic(args.config + "_hocbf", ("k_lattice_filter_hocbf", "k_lattice_filter_hocbf_rest"))
    traffic_adv = load_pmc_traffic(args.config, adv_kernels) if args.barrier == "reference" else traffic
    res = {
        "metric": METRIC,
        "value": solves / elapsed,
        "unit": "agent-QP solves/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "ms_per_step_with_stats": None if elapsed_stats is None else elapsed_stats / args.steps * 1e3,
        "ms_per_step_outputs_every_step": None if elapsed_hist is None else elapsed_hist / args.steps * 1e3,
        "outputs_every_step_note": "the timed steps replayed with every timestep's filtered control, status, nominal "
                                   "control and neighbour count stored (cbf_lattice_run_ex CBF_RUN_OUTPUT_HISTORY: "
                                   "the reference's per-step si_velocities); the headline run stores positions every "
                                   "timestep and the other outputs on each call's last timestep",
        "timed_region": "filter path only (stats=NULL); safety from a bit-identical statistics replay of the same "
                        "steps" if elapsed_stats is not None else "filter path with the statistics bookkeeping",
        "higher_is_better": True,
        "scaling": "weak" if args.weak and ws > 1 else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "end_state_sha256": state_sha,
        "config": {"workload": f"{args.config}: {W}x{rows_total} jittered lattice swarm (spacing {args.spacing}), "
                               + (f"lattice-Laplacian consensus (gain {args.gain})" if args.nominal is None else
                                  f"random-walk nominal control (amplitude {args.nominal[1]}, CBF_NOMINAL_RANDOM)")
                               + (" + radius-0.2 lattice-window cull" if cull == "window" else
                                  " + radius-0.2 cell-list cull")
                               + " + CBF QP + clip + Euler, one fused timestep per step",
                   "barrier": args.barrier,
                   "cull": cull,
                   "agents_total": n_total, "agents_per_gpu": n_local,
                   "parallelism": (f"row-stripe shards x{ws} ({rows} rows each), one {comm} "
                                   + ("all-to-all (ghost rows to the 2 neighbours + guard records to all)"
                                      if args.exchange == "neighbour" else "all-gather of ghost-row slabs")
                                   + f" per {k} steps ({halo * k} ghost rows per side)") if sharded else "single GPU",
                   "exchange_bytes_per_rank": S.exchange_bytes() if sharded else 0,
                   "solve_placement": ("inline in the filter" if solves_inline(S.params.c() if sharded else S.cp, rows * W)
                                       else "queued (k_lattice_filter_hard)")
                                      + (" (sharded: decided per sub-step window, its ghost rows included)"
                                         if sharded else ""),
                   "graph": use_graph,
                   "timesteps_per_call": max(plan) if chunk > 1 else 1},
        "timesteps_per_s": args.steps / elapsed,
        "solves_per_step": solves / args.steps,
        "exchange": exchange,
        "feasible_fraction": safety["feasible_fraction"] if safety else None,
        "safety": safety,
        "window_cull": window_cull,
        "full_size_check": check,
        "status_fraction_last_step": {"idle": codes[0] / len(status), "optimal": codes[1] / len(status),
                                      "relaxed": codes[2] / len(status),
                                      "box_infeasible": codes[3] / len(status)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic,
                     "kernel": (f"{adv_kernels[0].split('<')[0]}<f=0, no statistics> (the dominant kernel; "
                                + ("the start / stop events of its own launch (hipExtLaunchKernel), as a kernel trace "
                                   "times it" if own else "HIP events on its launch stream, the end event recorded "
                                   "by the advance call between it and the queued-QP kernel") + ")")
                     if args.barrier == "reference"
                     else "advance phase: k_lattice_filter_hocbf + k_lattice_filter_hocbf_rest",
                     "kernel_ms": f_ms,
                     "kernel_ms_stream_events": f_stream_ms,
                     "advance_phase": {"kernels": " + ".join(k.split("<")[0] for k in adv_kernels), "ms": k_ms,
                                       "achieved": achieved_adv, "frac": achieved_adv / HBM_PEAK_GBS,
                                       "traffic": traffic_adv},
                     "valu_busy": load_pmc_valu(args.config, adv_kernels[0]) if args.barrier == "reference" else None,
                     "valu_busy_2p4ghz": load_pmc_valu(args.config, adv_kernels[0], "valu_busy_2p4ghz")
                     if args.barrier == "reference" else None,
                     "valu_busy_note": "the dominant kernel's VALU issue fraction (rocprofv3 SQ_ACTIVE_INST_VALU, "
                                       "profiles/pmc_summary.json) over GRBM_GUI_ACTIVE / 8 cycles (reads high on "
                                       "short dispatches) and, valu_busy_2p4ghz, over its traced duration at the "
                                       "2.4 GHz peak clock (a lower bound): beside the HBM fraction, the limit it "
                                       "works against",
                     "algorithmic_bytes_per_launch": FILTER_BYTES_PER_AGENT * n_local,
                     "step_algorithmic_GBps": STEP_BYTES_PER_AGENT * n_local * args.steps / elapsed / 1e9 / ws},
    }
    return res


def exact_qp_regime(args):
    """cfg4r inside the default cfg4 line: the same 1M-agent lattice at spacing 0.22 with the
    random-walk nominal control (CBF_NOMINAL_RANDOM), the same --steps / --warmup, its own timed
    region -- the regime where most QPs are feasible with a binding row, i.e. where the reference
    (cbf.py:75-92) defines the answer.  `value` stays cfg4's; this record is beside it."""
    import copy
    a = copy.copy(args)
    a.config, a.spacing, a.nominal = "cfg4r", 0.22, ("random", 1.0, args.seed)
    r = bench_lattice(a, 1, 0, 0)
    sf = r["safety"]
    return {"config": "cfg4r", "workload": r["config"]["workload"], "value": r["value"], "unit": r["unit"],
            "ms_per_step": r["ms_per_step"], "ms_per_step_with_stats": r["ms_per_step_with_stats"],
            "steps": a.steps, "warmup": a.warmup, "timesteps_per_s": r["timesteps_per_s"],
            "feasible_fraction": sf["feasible_fraction"], "binding_fraction": sf["binding_fraction"],
            "relaxed_fraction": sf["relaxed_fraction"], "seidel_fraction": sf["seidel_fraction"],
            "max_violation_optimal": sf["max_violation_optimal"],
            "full_size_check": r["full_size_check"], "end_state_sha256": r["end_state_sha256"],
            "roofline": {k: r["roofline"][k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                          "kernel_ms", "advance_phase")},
            "note": "the exact-QP regime timed by the same command (bench.py --config cfg4r alone gives the same "
                    "line); no CPU baseline here (profiles/r0*_bench_cfg4r.json carry one)"}


def feasible_regime(args):
    """cfg4f inside the default cfg4 line: the same 1M-agent consensus lattice at spacing 0.2 (the
    window cull, as cfg4), the same --steps / --warmup, its own timed region.  Most of its QPs are
    feasible, so this is the branch of cbf.py:75-87 whose answer the reference defines (cfg4's QPs
    are almost all RELAXED: the +1 retry rule, which the reference never reaches on them); its
    full-size oracle check is tests/test_gpu_parity.py::test_window_full_size_driver_timesteps_vs_oracle
    [cfg4f].  `value` stays cfg4's; this record is beside it."""
    import copy
    a = copy.copy(args)
    a.config, a.spacing, a.nominal = "cfg4f", 0.2, None
    r = bench_lattice(a, 1, 0, 0)
    sf = r["safety"]
    return {"config": "cfg4f", "workload": r["config"]["workload"], "value": r["value"], "unit": r["unit"],
            "ms_per_step": r["ms_per_step"], "ms_per_step_with_stats": r["ms_per_step_with_stats"],
            "steps": a.steps, "warmup": a.warmup, "timesteps_per_s": r["timesteps_per_s"],
            "feasible_fraction": sf["feasible_fraction"], "binding_fraction": sf["binding_fraction"],
            "relaxed_fraction": sf["relaxed_fraction"], "seidel_fraction": sf["seidel_fraction"],
            "max_violation_optimal": sf["max_violation_optimal"], "window_cull": r["window_cull"],
            "full_size_check": r["full_size_check"], "end_state_sha256": r["end_state_sha256"],
            "roofline": {k: r["roofline"][k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                          "kernel_ms", "advance_phase")},
            "note": "the feasible regime timed by the same command (bench.py --config cfg4f alone gives the same "
                    "line)"}


def bench_allpairs(args, ws, rank, local):
    """cfg3: N = width x rows jittered lattice, every pair tested (FP64-VALU bound); replicas for N > 1."""
    import torch
    from cbf_amd import scenarios, swarm
    W, H = args.width, args.rows
    L = swarm.LatticeSwarm(scenarios.lattice(W, H, seed=args.seed + rank), W, H, gain=scenarios.LATTICE_GAIN,
                           method="allpairs")
    L.capture()
    for _ in range(args.warmup):
        L.step()
    L.reset_solves()
    if ws > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        L.step()
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    solves = L.solves_total()
    elapsed, solves = _reduce(elapsed, solves, ws)
    n = W * H
    pairs = float(n) * n * args.steps * ws / elapsed
    return {"metric": METRIC, "value": solves / elapsed, "unit": "agent-QP solves/s", "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"cfg3: {W}x{H} jittered lattice, all-pairs cull (every pair tested)",
                       "agents_per_gpu": n, "parallelism": "replicas" if ws > 1 else "single GPU"},
            "timesteps_per_s": args.steps / elapsed, "pair_tests_per_s": pairs,
            "roofline": {"bound": "valu-fp32", "achieved": pairs * 6 / 1e12, "peak": 157.3, "unit": "TFLOP/s",
                         "frac": pairs * 6 / 1e12 / 157.3, "traffic": None, "kernel": "k_allpairs_partial",
                         "note": "every pair is screened in fp32 (2 sub, 1 mul, 1 fma, 1 min = 6 flops, FMA counted "
                                 "as 2) against the MI355X FP32 vector peak, which counts packed FMAs; the screen "
                                 "is non-packed (no packed min) and its VALU issue is ~80 % busy (DESIGN.md sec. 4, "
                                 "profiles/r01_allpairs_dpp_pmc.txt); candidates the screen passes are re-tested "
                                 "exactly in fp64 (neighbour sets bit-identical to the oracle)"}}


def bench_mc(args, ws, rank, local):
    """cfg5: batched Monte-Carlo rendezvous, scenarios sharded across ranks (strong scaling: the
    100k-scenario batch is split), no per-step traffic, totals combined by all-reduces at the end
    (cbf_amd/montecarlo.py)."""
    import torch
    from cbf_amd.montecarlo import MonteCarlo
    mc = MonteCarlo(args.mc_scenarios, 16, 16, seed=args.seed)
    # as cfg4: the timed rollouts compute no statistics (counters only); the safety record comes
    # from a replay of the same steps from a snapshot, checked bit-identical (--timed-stats: off)
    mc.collect_stats = args.timed_stats
    for _ in range(max(1, args.warmup)):  # the same launches as a timed step
        mc.run(args.mc_inner)
    torch.cuda.synchronize()
    snap = None if args.timed_stats else mc.snapshot()
    mc.reset_totals()

    def timed():
        if ws > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for _ in range(args.steps):
            mc.run(args.mc_inner)
        ev1.record()
        torch.cuda.synchronize()
        if ws > 1:
            torch.distributed.barrier()
        return time.perf_counter() - t0, ev0.elapsed_time(ev1) / args.steps

    elapsed, kernel_ms = timed()
    elapsed, _ = _reduce(elapsed, 0, ws)
    elapsed_stats = None
    if snap is not None:
        counts_timed = mc.totals()["calls"]
        end = mc.pos.clone()
        mc.restore(snap)
        mc.collect_stats = True
        mc.reset_totals()
        elapsed_stats, _ = timed()
        elapsed_stats, _ = _reduce(elapsed_stats, 0, ws)
        same = bool(torch.equal(end, mc.pos))
        if ws > 1:
            f = torch.tensor([0 if same else 1], dtype=torch.int32, device="cuda")
            torch.distributed.all_reduce(f)
            same = int(f[0]) == 0
        if not same or mc.totals()["calls"] != counts_timed:
            raise RuntimeError("cfg5: the statistics replay did not repeat the timed rollouts bit for bit")
    tot = mc.totals()
    scen_steps = args.mc_scenarios * args.mc_inner * args.steps
    return {"metric": METRIC, "value": tot["calls"] / elapsed, "unit": "agent-QP solves/s", "n_gpus": ws,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "ms_per_step_with_stats": None if elapsed_stats is None else elapsed_stats / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"cfg5: {args.mc_scenarios} independent 16+16 rendezvous scenarios, "
                                   f"{args.mc_inner} timesteps per step, scenario-sharded",
                       "parallelism": f"scenario shards x{ws}" if ws > 1 else "single GPU"},
            "scenario_timesteps_per_s": scen_steps / elapsed,
            "feasible_fraction": tot["feasible_fraction"],
            "safety": {"solves": tot["calls"], "feasible_fraction": tot["feasible_fraction"],
                       "relaxed_fraction": tot["relaxed"] / max(tot["calls"], 1),
                       "box_infeasible": tot["box_infeasible"], "relax_cap": tot["relax_cap"],
                       "max_violation_optimal": tot["max_violation_optimal"],
                       "max_violation_original_rows_relaxed": tot["max_violation_original_rows_relaxed"],
                       "min_pairwise_distance": tot["min_pairwise_distance"]},
            "roofline": mc_roofline(kernel_ms, args.mc_scenarios // ws, args.mc_inner)}


def mc_roofline(kernel_ms, n_scen, inner):
    """cfg5's kernel keeps every scenario in LDS for the whole rollout (no HBM traffic per step), so
    its bound is the VALU: the VALU busy fraction of k_mc_rollout from the committed rocprof
    counters (profiles/pmc_summary.json "cfg5", tools/summarize_profile.py: SQ_ACTIVE_INST_VALU x 4 /
    (SIMDs x GRBM_GUI_ACTIVE)), measured on the same launch shape."""
    d = load_pmc("cfg5")   # the timed instantiation: f = 0, no statistics
    e = d.get("k_mc_rollout<true, false>", d.get("k_mc_rollout<true>", {}))
    out = {"bound": "valu", "unit": "fraction of VALU issue cycles", "peak": 1.0,
           "kernel": "k_mc_rollout<f=0, no statistics>",
           "kernel_ms": kernel_ms, "traffic": None}
    busy = e.get("valu_busy")
    out.update(achieved=busy, frac=busy,
               source="profiles/pmc_summary.json cfg5 (rocprofv3 --pmc, tools/profile.sh)" if busy is not None
               else "not profiled")
    return out


def cert_scenarios(B, N, seed=0):
    """Certificate workload: B independent scenarios of N agents on a jittered ring of radius
    min(0.05 N, 0.8) (inside the arena, neighbours >= 0.15 apart), each agent commanded toward
    the centre (pair rows bind, as in a rendezvous)."""
    rng = np.random.default_rng(seed)
    th = np.arange(N) * (2 * np.pi / N)
    rad = min(0.05 * N, 0.8)
    x = np.stack([rad * np.cos(th), rad * np.sin(th)], axis=1)[None] + rng.normal(0, 0.02, (B, N, 2))
    dxi = -x * rng.uniform(0.5, 2.0, (B, 1, 1))
    return np.ascontiguousarray(dxi), np.ascontiguousarray(x)


def cpu_baseline_cert(dxi, x, budget_s):
    """rps's CPU path for the certificate: the QP of barrier_certificates.py solved by the
    restated cvxopt coneqp with the options rps sets (reltol = feastol = 1e-2, maxiters 50;
    upstream, unverified) on a bounded sample, one core."""
    from oracle import cvxqp, rps_lite as R
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < budget_s and done < dxi.shape[0]:
        y, A, b = R.si_barrier_qp(dxi[done].T, x[done].T, safety_radius=0.12)
        n = y.shape[0]
        cvxqp.coneqp(2 * np.eye(n), -2 * y, A, b, maxiters=50, reltol=1e-2, feastol=1e-2)
        done += 1
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "certificate QPs/s", "cores": 1, "kind": "port",
            "sample": f"{done} scenarios of the same workload: rps's QP assembly + cvxopt coneqp restated in numpy "
                      f"(rps options), {dt:.1f} s on one core; rps and cvxopt are absent from the image"}


def bench_cert(args, ws, rank, local):
    """the coupled single-integrator barrier certificate (cross_and_rescue.py:163),
    batched over independent scenarios (scenario-sharded across ranks, weak scaling)."""
    import torch
    from cbf_amd import rps
    B, N = args.cert_scenarios, args.cert_agents
    dxi, x = cert_scenarios(B, N, seed=args.seed + rank)
    D, X = torch.tensor(dxi, device="cuda"), torch.tensor(x, device="cuda")
    cert = rps.SiBarrierCert(safety_radius=0.12)
    for _ in range(max(1, args.warmup)):
        r = cert.batch(D, X, iters=True)
    if ws > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        r = cert.batch(D, X, iters=True)
    e1.record()
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    elapsed, _ = _reduce(time.perf_counter() - t0, 0, ws)
    st = r["status"].cpu().numpy()
    na = r["n_active"].cpu().numpy()
    it = r["iters"].cpu().numpy()
    total = B * ws * args.steps
    return {"metric": "certificate QPs/s (coupled si_barrier_cert, SURVEY 8f row 3)", "value": total / elapsed,
            "unit": "certificate QPs/s", "n_gpus": ws, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"{B} scenarios x {N} agents per GPU, rendezvous-shaped, exact Goldfarb-Idnani "
                                   f"solve of {N * (N - 1) // 2 + 4 * N} rows x {2 * N} variables per scenario",
                       "parallelism": f"scenario shards x{ws}" if ws > 1 else "single GPU"},
            "agent_velocities_per_s": total * N / elapsed,
            "kernel_ms": e0.elapsed_time(e1) / args.steps,
            "optimal_fraction": float((st == 1).mean()), "mean_active_rows": float(na.mean()),
            "mean_iterations": float(it.mean()),
            "roofline": {"bound": "latency (LDS + dependent Givens chains)", "achieved": None, "peak": None,
                         "unit": None, "frac": None, "traffic": None,
                         "note": "one wavefront per scenario; the factors live in LDS, HBM traffic is 48 B/agent"},
            "_cert_sample": (dxi[:512], x[:512])}


def _reduce(elapsed, solves, ws):
    if ws == 1:
        return elapsed, solves
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    s = torch.tensor([solves], dtype=torch.int64, device="cuda")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    torch.distributed.all_reduce(s)
    return float(t[0]), int(s[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4", choices=["cfg4", "cfg4f", "cfg4r", "cfg3", "cfg5", "cert"],
                    help="cfg4f: the cfg4 swarm at spacing 0.2 (= dmin), where most QPs are feasible; cfg4r: "
                         "spacing 0.22 with random-walk nominal controls (amplitude 1), where most QPs are "
                         "feasible AND a barrier row binds (the exact QP path at scale)")
    ap.add_argument("--spacing", type=float, default=None, help="lattice spacing (cfg4 0.145, cfg4f 0.2)")
    ap.add_argument("--gain", type=float, default=None, help="lattice consensus gain (default 0.25)")
    ap.add_argument("--cert-scenarios", type=int, default=100000)
    ap.add_argument("--cert-agents", type=int, default=16)
    ap.add_argument("--mc-scenarios", type=int, default=100000)
    ap.add_argument("--mc-inner", type=int, default=10, help="cfg5: timesteps per bench step")
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks, one per GPU (without torchrun, bench.py starts them itself)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=1024,
                    help="lattice rows: of the whole lattice, split over the ranks (strong scaling, default), "
                         "or per rank with --weak")
    ap.add_argument("--weak", action="store_true", help="weak scaling: --rows rows per rank")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--eager", action="store_true", help="no hipGraph capture")
    ap.add_argument("--timed-stats", action="store_true",
                    help="cfg4: keep the rollout statistics inside the timed region (default: a bit-identical "
                         "statistics replay after it)")
    ap.add_argument("--kernel-iters", type=int, default=20)
    ap.add_argument("--chunk", type=int, default=50,
                    help="timesteps per cbf_lattice_run call (single-GPU graph path; 1 = one cbf_lattice_step per step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-exact-qp", action="store_true",
                    help="cfg4 single GPU: skip the feasible_regime / exact_qp_regime records (cfg4f, cfg4r timed "
                         "beside the headline)")
    ap.add_argument("--cull", default="auto", choices=["auto", "cells", "window"],
                    help="single-GPU lattice cull: auto = the lattice-window cull for the consensus lattice "
                         "(cfg4, cfg4f), the cell list for cfg4r's random walk")
    ap.add_argument("--barrier", default="reference", choices=["reference", "euclidean_hocbf"],
                    help="cfg4 single-GPU: the reference's L1 barrier rows or the Euclidean HOCBF mode")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds per CPU-baseline process and shape")
    ap.add_argument("--cpu-procs", type=int, default=None,
                    help="CPU-baseline processes (default: this job's host cores, oracle/cpu_baseline.py)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL; gloo = host-staged rehearsal, which "
                         "may put several ranks on one GPU)")
    ap.add_argument("--exchange", default="neighbour", choices=["neighbour", "allgather"],
                    help="sharded cfg4: ghost rows by one all-to-all to the two neighbours (default) or by one "
                         "all-gather to every rank")
    ap.add_argument("--substeps", type=int, default=None,
                    help="sharded cfg4: timesteps per halo exchange (default: min(16 for stripes of <= 512 rows, "
                         "else 8, rows per rank / (2 halo)))")
    ap.add_argument("--rank-timeout", type=float, default=None,
                    help="--gpus N without a launcher: overall seconds before the ranks still running are "
                         "terminated and named (default: from --steps / --warmup and --collective-timeout)")
    ap.add_argument("--rank-grace", type=float, default=30.0,
                    help="--gpus N without a launcher: seconds the other ranks get after one fails")
    ap.add_argument("--collective-timeout", type=float, default=300.0,
                    help="N > 1: torch.distributed timeout (s) of every collective; a rank blocked on a dead "
                         "peer raises after it")
    ap.add_argument("--shard", action="store_true",
                    help="cfg4: run the sharded step (halo pack + collective + unpack) even on one rank")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: this process starts the ranks and relays rank 0's line (it never touches the GPU)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:],
                              args.rank_timeout if args.rank_timeout else default_rank_timeout(args),
                              args.rank_grace))
    ws, rank, local = _dist_env()
    if ws != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} from the launcher but --gpus {args.gpus}")
    from cbf_amd import scenarios as _sc
    if args.spacing is None:
        args.spacing = {"cfg4f": 0.2, "cfg4r": 0.22}.get(args.config, _sc.LATTICE_SPACING)
    args.nominal = ("random", 1.0, args.seed) if args.config == "cfg4r" else None
    if args.gain is None:
        args.gain = _sc.LATTICE_GAIN
    # stdout carries exactly one JSON line: everything else that writes to fd 1 (RCCL prints a
    # version banner at communicator init) goes to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    if ws > 1 or args.shard:
        # (gloo: a rehearsal of several ranks on fewer GPUs, exchanges staged through the host)
        ndev = torch.cuda.device_count()
        if ndev == 0:
            raise SystemExit(f"bench.py rank {rank}: no GPU visible")
        dev = local % ndev if args.backend == "gloo" else local
        torch.cuda.set_device(dev)
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()) if ws == 1 else "29533")
        import datetime
        tmo = datetime.timedelta(seconds=args.collective_timeout)
        progress(f"init_process_group({args.backend}) on cuda:{dev}")
        if args.backend == "gloo":
            torch.distributed.init_process_group("gloo", rank=rank, world_size=ws, timeout=tmo)
        else:
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank,
                                                 world_size=ws, timeout=tmo)
    else:
        torch.cuda.set_device(0)
    if args.config == "cfg3":
        if args.rows == 1024 and args.width == 1024:
            args.width = args.rows = 256
        res = bench_allpairs(args, ws, rank, local)
    elif args.config == "cfg5":
        res = bench_mc(args, ws, rank, local)
    elif args.config == "cert":
        res = bench_cert(args, ws, rank, local)
    else:
        res = bench_lattice(args, ws, rank, local)
        if args.config == "cfg4" and ws == 1 and not args.shard and args.barrier == "reference" and \
                not args.no_exact_qp:
            res["feasible_regime"] = feasible_regime(args)
            res["exact_qp_regime"] = exact_qp_regime(args)
            sf = res["safety"] or {}
            res["regime_note"] = (
                f"cfg4 (the headline): {100 * sf.get('relaxed_fraction', float('nan')):.1f} % of its agent-QPs are "
                "RELAXED -- infeasible as posed, solved by the reference's +1 retry rule (cbf.py:84-87), a branch "
                "cvxopt never reaches (it returns an arbitrary 'unknown' iterate), so its answer is this "
                "repository's definition; feasible_regime (cfg4f) and exact_qp_regime (cfg4r) time the same "
                "command where most QPs are feasible, the branch whose answer the reference defines")
    if rank == 0:
        sample = res.pop("_cert_sample", None)
        res["cpu_baseline"] = None
        if ws == 1 and not args.no_cpu_baseline:
            progress("CPU baseline (oracle/, after the timed region)")
            res["cpu_baseline"] = cpu_baseline_for(args, sample)
        json_out.write(json.dumps(res) + "\n")
        json_out.flush()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
