"""Where the FedProx training step's proximal-term time goes (r04, VERDICT
r03 next 6): bench next_rows' step (train_fedprox.py:113-136 shape: the
client's gradients zeroed, the one-node proximal term, its backward) on the
wrn16_8 C100 layout, split into host phases (perf_counter, no sync inside:
what the Python / autograd side costs) and the same step's GPU time (its
three launches back to back).  One JSON line.  Usage: prox_profile.py [REPS]
    prox_profile.py prof K   -> only the term's kernels, K times (rocprofv3
                                kernel trace / PMC passes, tools/prox_prof.sh)"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from feddct_amd.layout import BucketLayout  # noqa: E402
from feddct_amd.prox import proximal_term  # noqa: E402
from feddct_amd.workload import load_manifest  # noqa: E402


def main():
    prof = len(sys.argv) > 2 and sys.argv[1] == "prof"
    reps = int(sys.argv[2 if prof else 1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lay = BucketLayout.from_manifest(load_manifest("wrn16_8_c100"))
    client, glob = bench._param_module(lay, dev, 1), bench._param_module(lay, dev, 2)
    for _ in range(5):
        client.zero_grad(set_to_none=True)
        proximal_term(client, glob, flat_grads=True).backward()
    torch.cuda.synchronize()
    if prof:
        # bench next_rows' kernel-only leg: fa_prox_norms + fa_prox_grad (both
        # gradients overwritten: 24 B/param) over 4 rotated bucket sets
        import ctypes
        from feddct_amd import _lib
        term = client.__dict__["_fa_prox"][id(glob)]
        norms = torch.empty(max(1, term.plan.nseg), device=dev)
        total = torch.empty((), device=dev)
        one = torch.ones((), device=dev)
        sets = [(term.ca.f32.clone(), term.ga.f32.clone(), torch.empty_like(term.ca.f32),
                 torch.empty_like(term.ga.f32)) for _ in range(4)]
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        # beside them, a one-workgroup kernel that reads 256 B (the read
        # probe at n = 64): the floor of any single-workgroup launch, for
        # the finish's duration
        tiny = torch.ones(64, device=dev)
        sink = torch.zeros(256, device=dev)
        for i in range(reps):
            _lib.check(_lib.lib.fa_read_probe_f32(tiny.data_ptr(), 64, sink.data_ptr(), 0, st))
            a, b, ga, gb = sets[i % 4]
            _lib.check(_lib.lib.fa_prox_norms(term.plan.handle, a.data_ptr(), b.data_ptr(),
                                              norms.data_ptr(), total.data_ptr(), st))
            _lib.check(_lib.lib.fa_prox_grad(term.plan.handle, a.data_ptr(), b.data_ptr(),
                                             norms.data_ptr(), one.data_ptr(), 1.0,
                                             ga.data_ptr(), gb.data_ptr(), st))
        torch.cuda.synchronize()
        print(f"prox term kernels: {reps} steps, {lay.f32_numel} floats per bucket")
        return
    ph = {k: [] for k in ("zero_grad", "term_call", "backward", "step_host", "step_wall")}
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        client.zero_grad(set_to_none=True)
        t1 = time.perf_counter()
        pt = proximal_term(client, glob, flat_grads=True)
        t2 = time.perf_counter()
        pt.backward()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        for k, a, b in (("zero_grad", t0, t1), ("term_call", t1, t2), ("backward", t2, t3),
                        ("step_host", t0, t3), ("step_wall", t0, t4)):
            ph[k].append((b - a) * 1e6)
    out = {k: round(sorted(v)[len(v) // 2], 1) for k, v in ph.items()}
    # the same step's kernels back to back (bound term, no autograd)
    term = client.__dict__["_fa_prox"][id(glob)]
    gout = torch.ones((), device=dev)

    def kernels():
        term.norms_forward()
        term.accumulate_grads(gout)
    t, _ = bench.timed_launches(kernels, reps, 5)
    out["kernels_us"] = round(t * 1e6, 1)
    # the pieces of the term call, host side
    sub = {k: [] for k in ("lookup_valid", "apply")}
    from feddct_amd.prox import _ProxFlat
    for _ in range(reps):
        t0 = time.perf_counter()
        cache = client.__dict__["_fa_prox"]
        t_ = cache[id(glob)]
        ok = t_.valid()
        t1 = time.perf_counter()
        _, anchor, _ = t_._flat_state()
        r = _ProxFlat.apply(t_, anchor)
        t2 = time.perf_counter()
        assert ok
        sub["lookup_valid"].append((t1 - t0) * 1e6)
        sub["apply"].append((t2 - t1) * 1e6)
        del r
    out.update({k: round(sorted(v)[len(v) // 2], 1) for k, v in sub.items()})
    # the host side of the term's own work, no autograd: forward launches,
    # backward launch + gradient binding
    sub = {k: [] for k in ("norms_forward_host", "accumulate_grads_host")}
    for _ in range(reps):
        torch.cuda.synchronize()
        client.zero_grad(set_to_none=True)
        t0 = time.perf_counter()
        term.norms_forward()
        t1 = time.perf_counter()
        term.accumulate_grads(gout)
        t2 = time.perf_counter()
        sub["norms_forward_host"].append((t1 - t0) * 1e6)
        sub["accumulate_grads_host"].append((t2 - t1) * 1e6)
    out.update({k: round(sorted(v)[len(v) // 2], 1) for k, v in sub.items()})

    # autograd's own price for ONE Python Function node on a CUDA tensor: a
    # node that does nothing, forward + backward (what any one-node Python
    # form pays on top of its work)
    class Nop(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.new_empty(())

        @staticmethod
        def backward(ctx, g):
            return None
    anchor = torch.zeros((), device=dev, requires_grad=True)
    sub = {k: [] for k in ("nop_apply", "nop_backward")}
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        y = Nop.apply(anchor)
        t1 = time.perf_counter()
        y.backward()
        t2 = time.perf_counter()
        sub["nop_apply"].append((t1 - t0) * 1e6)
        sub["nop_backward"].append((t2 - t1) * 1e6)
    out.update({k: round(sorted(v)[len(v) // 2], 1) for k, v in sub.items()})
    # and the optimizer's zero_grad on a plain module of the same 100 params
    plain = torch.nn.ParameterList([torch.nn.Parameter(p.detach().clone())
                                    for p in client.parameters()])
    for p in plain:
        p.grad = torch.zeros_like(p)
    zs = []
    for _ in range(reps):
        for p in plain:
            p.grad = torch.zeros_like(p) if p.grad is None else p.grad
        t0 = time.perf_counter()
        plain.zero_grad(set_to_none=True)
        zs.append((time.perf_counter() - t0) * 1e6)
    out["zero_grad_plain_params_us"] = round(sorted(zs)[len(zs) // 2], 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
