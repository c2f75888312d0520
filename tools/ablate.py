"""A/B harness for the lattice step kernels: builds variants of libcbf_amd.so with compile-time
switches and times cbf_lattice_build / cbf_lattice_advance of each, interleaved in one process
(HIP events on the launch stream).

  python tools/ablate.py build            # in the build container (hipcc)
  python tools/ablate.py run [--rounds R] # on the GPU box
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_ablate")
SETS = {}
SETS["allpairs"] = {
    "ap_lds_diff": [],
    "ap_lds_expand": ["-DCBF_AP_EXPAND=1"],
    "ap_lds_diff_packed": ["-DCBF_AP_PACKED=1"],
    "ap_dpp": ["-DCBF_AP_DPP=1", "-DCBF_AP_EXPAND=1"],
    "ap_dpp_diff": ["-DCBF_AP_DPP=1"],
}
SETS["hardinline"] = {
    "queue": [],
    "inline": ["-DCBF_HARD_INLINE=1"],
}
SETS["nominal"] = {
    "in_scatter": [],
    "in_bin": ["-DCBF_NOMINAL_IN_SCATTER=0"],
}
SETS["head"] = {"tree": []}
SETS["hsort"] = {"reg": [], "insertion": ["-DCBF_HSORT_REG=0"]}
SETS["nt"] = {"plain": [], "nt": ["-DCBF_NT_STORES=1"]}
SETS["wide"] = {"w1024": [], "w256": ["-DCBF_WIDE_BLOCKS=256"], "w128": ["-DCBF_WIDE_BLOCKS=128"]}
SETS["hcert"] = {"nocert": [], "cert": ["-DCBF_HOCBF_CERT=1"]}
SETS["scan"] = {"sumagg": [], "lookback": ["-DCBF_SCAN_SUMAGG=0"]}
SETS["scanst"] = {"vst": [], "scalar": ["-DCBF_SCAN_VST=0"]}
SETS["scanper"] = {"per8": [], "per16": ["-DCBF_SCAN_PER=16"], "per4": ["-DCBF_SCAN_PER=4"]}
SETS["phases"] = {
    "full": [],
    "no_qp": ["-DCBF_ABLATE=1"],
    "no_qp_no_rows": ["-DCBF_ABLATE=2"],
    "no_scan": ["-DCBF_ABLATE=3"],
}
SETS["flush"] = {
    "full": [],
    "pushbf": ["-DCBF_PUSH_BF=1"],
    "bqlds": ["-DCBF_BQ_LDS=1"],
    "both": ["-DCBF_PUSH_BF=1", "-DCBF_BQ_LDS=1"],
    "both_f2": ["-DCBF_PUSH_BF=1", "-DCBF_BQ_LDS=1", "-DCBF_FLUSH_U=2"],
    "both_s8": ["-DCBF_PUSH_BF=1", "-DCBF_BQ_LDS=1", "-DCBF_SCAN_U=8"],
}
SETS["scan32"] = {
    "full": [],
    "s32": ["-DCBF_SCAN32=1"],
    "s32_bq": ["-DCBF_SCAN32=1", "-DCBF_BQ_LDS=1"],
    "s32_bq_s8": ["-DCBF_SCAN32=1", "-DCBF_BQ_LDS=1", "-DCBF_SCAN_U=8"],
    "s32_bq_bf": ["-DCBF_SCAN32=1", "-DCBF_BQ_LDS=1", "-DCBF_PUSH_BF=1"],
    "bq": ["-DCBF_BQ_LDS=1"],
}
SETS["hard"] = {
    "full": [],
    "hard64": ["-DCBF_HARD_BLOCKS=64"],
    "hard128": ["-DCBF_HARD_BLOCKS=128"],
    "hard1024": ["-DCBF_HARD_BLOCKS=1024"],
}
SETS["xcd"] = {
    "full": [],
    "noxcd": ["-DCBF_XCD_REMAP=0"],
}
SETS["stage"] = {
    "full": [],
    "stage": ["-DCBF_LDS_STAGE=1"],
    "stage2": ["-DCBF_LDS_STAGE=2"],
}
SETS["mask"] = {
    "full": [],
    "mask": ["-DCBF_HIT_MASK=1"],
    "mask_f2": ["-DCBF_HIT_MASK=1", "-DCBF_FLUSH_U=2"],
    "mask_s8": ["-DCBF_HIT_MASK=1", "-DCBF_SCAN_U=8"],
}
SETS["inline"] = {
    "full": [],
    "inline4": ["-DCBF_SCAN_INLINE=1"],
    "inline3": ["-DCBF_SCAN_INLINE=1", "-DCBF_INLINE_U=3"],
    "inline6": ["-DCBF_SCAN_INLINE=1", "-DCBF_INLINE_U=6"],
}
SETS["occ"] = {
    "full": [],
    "cap12": ["-DCBF_HIT_CAP=12"],
    "cap10_w8": ["-DCBF_HIT_CAP=10", "-DCBF_FILTER_WPE=8"],
    "cap12_w7": ["-DCBF_HIT_CAP=12", "-DCBF_FILTER_WPE=7"],
    "cap16_nobq_w8": ["-DCBF_BQ_LDS=0", "-DCBF_FILTER_WPE=8"],
    "cap10_nobq_w8": ["-DCBF_HIT_CAP=10", "-DCBF_BQ_LDS=0", "-DCBF_FILTER_WPE=8"],
}
SETS["mc"] = {
    "mc_base": [],
    "mc_screen": ["-DCBF_MC_SCREEN=1"],
    "mc_easy": ["-DCBF_MC_EASY=1"],
    "mc_both": ["-DCBF_MC_SCREEN=1", "-DCBF_MC_EASY=1"],
}
SETS["ext"] = {
    "block64": [],
    "wave64": ["-DCBF_EXT_WAVE=1"],
    "wave512": ["-DCBF_EXT_WAVE=1", "-DCBF_EXT_SLOTS=512"],
    "block16": ["-DCBF_EXT_SLOTS=16"],
}
VARIANTS = {
    "full": [],
    "flush2": ["-DCBF_FLUSH_U=2"],
    "flush4": ["-DCBF_FLUSH_U=4"],
    "scan6": ["-DCBF_SCAN_U=6"],
    "scan8": ["-DCBF_SCAN_U=8"],
    "scan8_flush2": ["-DCBF_SCAN_U=8", "-DCBF_FLUSH_U=2"],
    "scan6_flush4": ["-DCBF_SCAN_U=6", "-DCBF_FLUSH_U=4"],
}


def _variants():
    """Compile-time ablations of the working tree (the set named by ABLATE_SET, else VARIANTS)
    plus `rev_<git rev>` builds listed in tools/_ablate/revs (one revision per line), so a change
    can be A/B-timed against an earlier commit in the same process."""
    rf = os.path.join(OUT, "revs")
    revs = open(rf).read().split() if os.path.exists(rf) else []
    sel = SETS[os.environ["ABLATE_SET"]] if os.environ.get("ABLATE_SET") else VARIANTS
    v = {k: (None, d) for k, d in sel.items()}
    v.update({f"rev_{rev}": (rev, []) for rev in revs})
    return v


def build(revs=()):
    from cbf_amd import build as B
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "revs"), "w") as f:
        f.write("\n".join(revs))
    for name, (rev, defs) in _variants().items():
        csrc, inc = B.CSRC, os.path.join(ROOT, "include")
        if rev is not None:
            src_root = os.path.join(OUT, f"src_{rev}")
            os.makedirs(src_root, exist_ok=True)
            arc = subprocess.run(["git", "-C", ROOT, "archive", rev, "cbf_amd/csrc", "include"], check=True,
                                 capture_output=True).stdout
            subprocess.run(["tar", "-x", "-C", src_root], input=arc, check=True)
            csrc, inc = os.path.join(src_root, "cbf_amd", "csrc"), os.path.join(src_root, "include")
        flags = [f for f in B.FLAGS if f not in (B.CSRC, os.path.join(ROOT, "include"))]
        flags = [x for x in flags if x != "-I"] + ["-I", inc, "-I", csrc]
        objs = []
        for src in B.SOURCES:
            o = os.path.join(OUT, f"{name}_{os.path.splitext(src)[0]}.o")
            lang = ["-x", "hip"] if src.endswith(".hip") else []
            subprocess.run([B.HIPCC] + flags + defs + lang + ["-c", os.path.join(csrc, src), "-o", o], check=True)
            objs.append(o)
        subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-o", os.path.join(OUT, f"lib_{name}.so")]
                       + objs, check=True)
        print("built", name)


def run(rounds, iters, W, H):
    import numpy as np
    import torch
    from cbf_amd import _lib, scenarios, swarm
    torch.cuda.set_device(0)
    libs = {}
    names = list(_variants())
    for name in names:
        L = C.CDLL(os.path.join(OUT, f"lib_{name}.so"))
        for fn, (res, args) in _lib.SIGNATURES.items():
            getattr(L, fn).restype = res
            getattr(L, fn).argtypes = args
        libs[name] = L
    pos0 = scenarios.lattice(W, H, seed=0)
    grid = swarm.grid_for_points(pos0, 0.2)
    cp = _lib.make_params(15)
    hp = _lib.CbfHocbf(1.0, 1.0)
    ws_bytes = max(L.cbf_lattice_workspace_size(W, H, C.byref(grid)) for L in libs.values())
    st = {}
    for name in names:
        st[name] = dict(pos=torch.tensor(pos0, device="cuda"), vel=torch.empty((W * H, 2), dtype=torch.float64,
                                                                                device="cuda"),
                        u=torch.empty((W * H, 2), dtype=torch.float64, device="cuda"),
                        status=torch.empty(W * H, dtype=torch.int32, device="cuda"),
                        cnt=torch.empty(W * H, dtype=torch.int32, device="cuda"),
                        ws=torch.zeros(ws_bytes, dtype=torch.uint8, device="cuda"))
    P = _lib.ptr
    times = {n: {"build": [], "advance": []} for n in names}
    for r in range(rounds):
        for name, L in libs.items():
            s = st[name]
            for _ in range(iters):
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record()
                _lib.check(L.cbf_lattice_build(cp, C.byref(grid), W, H, 0, H, 0, H, P(s["pos"]), 0.25, P(s["vel"]),
                                               P(s["ws"]), ws_bytes, _lib.stream_handle()), "build")
                e1.record()
                if os.environ.get("ABLATE_HOCBF"):  # the Euclidean HOCBF advance instead
                    _lib.check(L.cbf_lattice_advance_hocbf(cp, C.byref(hp), C.byref(grid), W, H, 0, H, 0, H,
                                                           P(s["pos"]), 1 / 30, P(s["pos"]), P(s["u"]),
                                                           P(s["status"]), P(s["cnt"]), 0, None, None, P(s["ws"]),
                                                           ws_bytes, _lib.stream_handle()), "advance_hocbf")
                else:
                    _lib.check(L.cbf_lattice_advance(cp, C.byref(grid), W, H, 0, H, 0, H, P(s["pos"]), 1 / 30,
                                                     P(s["pos"]), P(s["u"]), P(s["status"]), P(s["cnt"]), 0, None,
                                                     None, P(s["ws"]), ws_bytes, _lib.stream_handle()), "advance")
                e2.record()
                torch.cuda.synchronize()
                if r > 0:
                    times[name]["build"].append(e0.elapsed_time(e1))
                    times[name]["advance"].append(e1.elapsed_time(e2))
    res = {n: {k: {"median_us": float(np.median(v)) * 1e3, "min_us": float(np.min(v)) * 1e3}
               for k, v in t.items()} for n, t in times.items()}
    # every variant ran the same number of steps from the same state: results must be bit-identical
    ref = names[0]
    for n in names[1:]:
        same = all(torch.equal(st[n][f], st[ref][f]) for f in ("pos", "vel", "u", "status", "cnt"))
        res[n]["bit_identical_to_" + ref] = bool(same)
        if not same:
            print(f"MISMATCH {n} vs {ref}", file=sys.stderr)
    print(json.dumps(res, indent=1))
    return res


def run_shard(rounds, iters, W, H, k=4):
    """The sharded step at one rank (cbf_halo_pack every k sub-steps + cbf_lattice_step_sharded),
    per variant, against the plain cbf_lattice_step; results checked bit-for-bit."""
    import numpy as np
    import torch
    from cbf_amd import _lib, scenarios, swarm
    torch.cuda.set_device(0)
    libs = {}
    names = list(_variants())
    for name in names:
        L = C.CDLL(os.path.join(OUT, f"lib_{name}.so"))
        for fn, (res, args) in _lib.SIGNATURES.items():
            getattr(L, fn).restype = res
            getattr(L, fn).argtypes = args
        libs[name] = L
    pos0 = scenarios.lattice(W, H, seed=0)
    grid = swarm.grid_for_points(pos0, 0.2)
    cp = _lib.make_params(15)
    P = _lib.ptr
    st = {}
    for name, L in libs.items():
        wsb = L.cbf_lattice_workspace_size(W, H, C.byref(grid))
        kb = L.cbf_halo_ext_bytes(k)
        d = dict(pos=torch.tensor(pos0, device="cuda"), vel=torch.empty((W * H, 2), dtype=torch.float64, device="cuda"),
                 u=torch.empty((W * H, 2), dtype=torch.float64, device="cuda"),
                 status=torch.empty(W * H, dtype=torch.int32, device="cuda"),
                 cnt=torch.empty(W * H, dtype=torch.int32, device="cuda"),
                 ws=torch.zeros(wsb, dtype=torch.uint8, device="cuda"), wsb=wsb,
                 keys=torch.empty(kb // 8, dtype=torch.int64, device="cuda"),
                 send=torch.zeros(2 * 16 * W * 2 + 8 * k, dtype=torch.float64, device="cuda"),
                 solves=torch.zeros(1024, dtype=torch.int64, device="cuda"))
        _lib.check(L.cbf_halo_ext_reset(P(d["keys"]), k, _lib.stream_handle()), "reset")
        st[name] = d
    times = {n: [] for n in names}
    for r in range(rounds):
        for name, L in libs.items():
            d = st[name]
            sw = L.cbf_halo_ext_bytes(1) // 8
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for it in range(iters):
                s = it % k
                if s == 0:
                    _lib.check(L.cbf_halo_pack(W, 16, W * H, P(d["pos"]), P(d["keys"]), k, P(d["send"]),
                                               _lib.stream_handle()), "pack")
                _lib.check(L.cbf_lattice_step_sharded(cp, C.byref(grid), W, H, 0, H, 0, H, 0, H, P(d["pos"]), 0.25,
                                                      1 / 30, P(d["pos"]), P(d["vel"]), P(d["u"]), P(d["status"]),
                                                      P(d["cnt"]), 3, P(d["keys"][s * sw:]), P(d["solves"]),
                                                      P(d["ws"]), d["wsb"], _lib.stream_handle()), "step")
            e1.record()
            torch.cuda.synchronize()
            if r > 0:
                times[name].append(e0.elapsed_time(e1) / iters)
    res = {n: {"us_per_step": float(np.median(v)) * 1e3} for n, v in times.items()}
    ref = names[0]
    for n in names[1:]:
        for f in ("pos", "u", "status", "send"):
            res[n][f"{f}_identical"] = bool(torch.equal(st[n][f], st[ref][f]))
        res[n]["send_ext"] = st[n]["send"][-8 * k:].view(k, 8)[:, :6].tolist()
    res[ref]["send_ext"] = st[ref]["send"][-8 * k:].view(k, 8)[:, :6].tolist()
    print(json.dumps(res, indent=1))


def run_mc(rounds, iters, n_scen=100000, steps=10):
    """cbf_mc_rollout (cfg5 shape) per variant; final positions and counters checked bit-for-bit."""
    import numpy as np
    import torch
    from cbf_amd import _lib, scenarios
    torch.cuda.set_device(0)
    names = list(_variants())
    libs = {}
    for name in names:
        L = C.CDLL(os.path.join(OUT, f"lib_{name}.so"))
        for fn, (res, args) in _lib.SIGNATURES.items():
            getattr(L, fn).restype = res
            getattr(L, fn).argtypes = args
        libs[name] = L
    pos0 = torch.tensor(scenarios.mc_scenarios(n_scen, 16, 16, seed=0), device="cuda")
    cp = _lib.make_params(15)
    P = _lib.ptr
    th = -np.pi / 16
    st = {n: dict(pos=pos0.clone(), cnt=torch.zeros((n_scen, 4), dtype=torch.int64, device="cuda"),
                  mv=torch.zeros(n_scen, dtype=torch.float64, device="cuda")) for n in names}
    times = {n: [] for n in names}
    for r in range(rounds):
        for name, L in libs.items():
            d = st[name]
            for _ in range(iters):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                _lib.check(L.cbf_mc_rollout(cp, n_scen, 16, 16, steps, 1 / 30, float(np.cos(th)), float(np.sin(th)),
                                            1.0, scenarios.MC_GAIN, P(d["pos"]), P(d["cnt"]), P(d["mv"]),
                                            _lib.stream_handle()), "mc")
                b.record()
                torch.cuda.synchronize()
                if r > 0:
                    times[name].append(a.elapsed_time(b))
    res = {n: {"ms_per_call": float(np.median(v))} for n, v in times.items()}
    ref = names[0]
    for n in names[1:]:
        res[n]["bit_identical"] = bool(all(torch.equal(st[n][f], st[ref][f]) for f in ("pos", "cnt", "mv")))
    print(json.dumps(res, indent=1))


def run_allpairs(rounds, iters, W, H):
    import numpy as np
    import torch
    from cbf_amd import _lib, scenarios
    torch.cuda.set_device(0)
    names = list(_variants())
    libs = {}
    for name in names:
        L = C.CDLL(os.path.join(OUT, f"lib_{name}.so"))
        for fn, (res, args) in _lib.SIGNATURES.items():
            getattr(L, fn).restype = res
            getattr(L, fn).argtypes = args
        libs[name] = L
    pos = torch.tensor(scenarios.lattice(W, H, seed=0), device="cuda")
    vel = torch.randn(W * H, 2, dtype=torch.float64, device="cuda") * 0.05
    n = W * H
    u = torch.empty(n, 2, dtype=torch.float64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    cp = _lib.make_params(15)
    P = _lib.ptr
    ws = {name: torch.empty(L.cbf_allpairs_workspace_size(n, n), dtype=torch.uint8, device="cuda")
          for name, L in libs.items()}
    ref = None
    times = {k: [] for k in names}
    for r in range(rounds):
        for name, L in libs.items():
            for _ in range(iters):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                _lib.check(L.cbf_filter_allpairs_split(cp, n, 0, P(pos), P(vel), 0, n, P(u), P(st), None,
                                                       P(ws[name]), ws[name].numel(), _lib.stream_handle()),
                           "allpairs_split")
                b.record()
                torch.cuda.synchronize()
                if r > 0:
                    times[name].append(a.elapsed_time(b))
            if ref is None:
                ref = u.clone()
            if not torch.equal(u, ref):
                bad = (u != ref).any(1)
                print(f"MISMATCH {name}: {int(bad.sum())} egos, max |du| {float((u - ref).abs().max())}",
                      file=sys.stderr)
    res = {k: {"median_us": float(np.median(v)) * 1e3, "pair_tests_per_s": n * n / (float(np.median(v)) * 1e-3)}
           for k, v in times.items()}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run", "run_allpairs", "run_shard", "run_mc"])
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--W", type=int, default=1024)
    ap.add_argument("--H", type=int, default=1024)
    ap.add_argument("--revs", nargs="*", default=[], help="build: also build these git revisions")
    a = ap.parse_args()
    if a.cmd == "build":
        build(a.revs)
    elif a.cmd == "run_allpairs":
        run_allpairs(a.rounds, a.iters, a.W, a.H)
    elif a.cmd == "run_shard":
        run_shard(a.rounds, a.iters, a.W, a.H)
    elif a.cmd == "run_mc":
        run_mc(a.rounds, a.iters)
    else:
        run(a.rounds, a.iters, a.W, a.H)
