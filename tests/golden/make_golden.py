"""Generate the committed golden fixtures by running the REFERENCE.

Run in the build container only (``/root/reference`` does not exist on the GPU
box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own ``server_aggregate`` from train_fedavg.py
(:138-149), train_fedprox.py (:143-154), train_feddct.py (:34-56) and
train_splitfed.py (:34-56) plus its model code (model/splitnet.py,
model/splitnetsl.py), stubbing only the logging/data imports those scripts
pull in at module level and never use on this path (tensorboardX,
setproctitle, torchvision, cv2 ...).  Nothing from the reference is copied:
the outputs written here are data.

Outputs
  feddct_amd/manifests/<layout>.json  key/shape/dtype of each model layout
  tests/golden/small_goldens.npz      reference outputs on PRNG inputs (small)
  tests/golden/digests.json           SHA-256 of reference outputs, full size
"""
from __future__ import annotations

import argparse
import hashlib
import importlib.abc
import importlib.machinery
import json
import os
import sys
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
sys.path.insert(0, REPO)

from feddct_amd import synth  # noqa: E402

STUB_ROOTS = {"setproctitle", "tensorboardX", "torchvision", "cv2",
              "albumentations", "skimage"}


class _Anything(types.ModuleType):
    """Module whose every attribute is a harmless callable/class."""

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return type(name, (), {"__init__": lambda self, *a, **k: None,
                               "__call__": lambda self, *a, **k: None})


class _StubFinder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, fullname, path, target=None):
        if fullname.split(".")[0] in STUB_ROOTS:
            return importlib.machinery.ModuleSpec(fullname, self, is_package=True)
        return None

    def create_module(self, spec):
        m = _Anything(spec.name)
        m.__path__ = []
        return m

    def exec_module(self, module):
        pass


def import_reference():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.meta_path.insert(0, _StubFinder())
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir("/tmp")
    try:
        import train_fedavg, train_fedprox, train_feddct, train_splitfed  # noqa
        from model import splitnet, splitnetsl  # noqa
        from params import train_params  # noqa
        from utils import norm  # noqa
    finally:
        os.chdir(cwd)
    return dict(fedavg=train_fedavg, fedprox=train_fedprox, feddct=train_feddct,
                splitfed=train_splitfed, splitnet=splitnet, splitnetsl=splitnetsl,
                train_params=train_params, norm=norm)


def ref_args(ref, argv):
    saved = sys.argv
    sys.argv = ["x"] + argv
    try:
        args = ref["train_params"].add_parser_params(argparse.ArgumentParser())
    finally:
        sys.argv = saved
    args.loop_factor = 1 if args.is_train_sep or args.is_single_branch else args.split_factor
    return args


def build_models(ref):
    """Reference model instances for each layout (CPU, random init)."""
    norm = ref["norm"]
    out = {}
    for nc, tag in ((10, "c10"), (100, "c100")):
        a = ref_args(ref, ["--arch", "wide_resnet16_8", "--split_factor", "1",
                           "--dataset", "cifar10" if nc == 10 else "cifar100",
                           "--num_classes", str(nc)])
        out[f"wrn16_8_{tag}"] = lambda a=a: ref["splitnet"].SplitNet(
            a, norm_layer=norm.norm(a.norm_mode), criterion=None)
        b = ref_args(ref, ["--arch", "wide_resnetsl16_8", "--split_factor", "4",
                           "--dataset", "cifar10" if nc == 10 else "cifar100",
                           "--num_classes", str(nc)])
        out[f"wrnsl16_8_sf4_{tag}_main"] = lambda b=b: ref["splitnetsl"].SplitNetMainClient(
            b, norm_layer=norm.norm(b.norm_mode), criterion=None)
        out[f"wrnsl16_8_sf4_{tag}_proxy"] = lambda b=b: ref["splitnetsl"].SplitNetProxyClient(
            b, norm_layer=norm.norm(b.norm_mode), criterion=None)
    return out


# The reference's other FedDCT sweep layouts (r03; VERDICT r02 missing 1):
# (arch, split_factor, num_selected) from the launch scripts, all CIFAR-100:
#   script/feddct_wrn168_split{2,8,16,32}_cifar100_96clients_96choose_650rounds.sh:27
#   script/feddct_resnet110_split4_cifar100_100clients_100choose_650rounds.sh:27  (N=25)
#   script/feddct_resnet110_split4_cifar100_80clients_80choose_650rounds.sh       (N=20)
SWEEP = [("wide_resnetsl16_8", "wrnsl16_8", 2, 48), ("wide_resnetsl16_8", "wrnsl16_8", 8, 12),
         ("wide_resnetsl16_8", "wrnsl16_8", 16, 6), ("wide_resnetsl16_8", "wrnsl16_8", 32, 3),
         ("resnet110sl", "resnet110sl", 4, 25), ("resnet110sl", "resnet110sl", 4, 20)]


def sweep_name(tag, sf):
    return f"{tag}_sf{sf}_c100"


def build_sweep_models(ref):
    norm = ref["norm"]
    out = {}
    for arch, tag, sf, _ in SWEEP:
        b = ref_args(ref, ["--arch", arch, "--split_factor", str(sf), "--dataset", "cifar100",
                           "--num_classes", "100"])
        name = sweep_name(tag, sf)
        out[name + "_main"] = lambda b=b: ref["splitnetsl"].SplitNetMainClient(
            b, norm_layer=norm.norm(b.norm_mode), criterion=None)
        out[name + "_proxy"] = lambda b=b: ref["splitnetsl"].SplitNetProxyClient(
            b, norm_layer=norm.norm(b.norm_mode), criterion=None)
    return out


def sweep_digests():
    """Manifests + reference FedDCT digests for SWEEP (merged into
    digests.json; the existing entries are left as they are)."""
    ref = import_reference()
    torch.set_num_threads(8)
    torch.manual_seed(0)
    builders = build_sweep_models(ref)
    man_dir = os.path.join(REPO, "feddct_amd", "manifests")
    manifests = {}
    for name, mk in builders.items():
        m = manifest_of(name, mk())
        manifests[name] = m
        with open(os.path.join(man_dir, name + ".json"), "w") as f:
            json.dump(m, f, indent=0)
        print(name, len(m["keys"]), "keys", flush=True)
    path = os.path.join(REPO, "tests", "golden", "digests.json")
    with open(path) as f:
        digests = json.load(f)
    for _, tag, sf, n in SWEEP:
        lm, lp = sweep_name(tag, sf) + "_main", sweep_name(tag, sf) + "_proxy"
        if f"feddct/{lp}/n{n}" in digests:
            continue
        gm, gp = builders[lm](), builders[lp]()
        ms = [builders[lm]() for _ in range(n)]
        ps = [builders[lp]() for _ in range(n)]
        for i in range(n):
            fill_module(ms[i], manifests[lm], i, synth.MODE_REALISTIC)
            fill_module(ps[i], manifests[lp], i, synth.MODE_REALISTIC)
        ref["feddct"].server_aggregate(gm, gp, ms, ps)
        digests[f"feddct/{lm}/n{n}"] = state_digest(gm)
        digests[f"feddct/{lp}/n{n}"] = state_digest(gp)
        print("feddct", lm, n, digests[f"feddct/{lm}/n{n}"], digests[f"feddct/{lp}/n{n}"],
              flush=True)
        del gm, gp, ms, ps
        with open(path, "w") as f:   # after every case: a long run keeps what it has
            json.dump(digests, f, indent=1)


def manifest_of(name, module):
    keys = []
    for k, v in module.state_dict().items():
        keys.append({"key": k, "shape": list(v.shape), "dtype": str(v.dtype).replace("torch.", "")})
    return {"name": name, "keys": keys}


def fill_module(module, manifest, client, mode):
    sd = module.state_dict()
    with torch.no_grad():
        for k, arr in synth.gen_state(manifest, client, mode):
            sd[k].copy_(torch.from_numpy(np.array(arr, copy=True)))


def state_digest(module):
    """SHA-256 over key order + raw little-endian bytes of every tensor."""
    h = hashlib.sha256()
    for k, v in module.state_dict().items():
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


class Holder(torch.nn.Module):
    """Small module holding fp32 parameters and 0-dim int64 buffers, in the
    key order of a synthetic manifest."""

    def __init__(self, manifest):
        super().__init__()
        self._names = []
        for i, e in enumerate(manifest["keys"]):
            nm = e["key"]
            if e["dtype"] == "int64":
                self.register_buffer(nm, torch.zeros(e["shape"], dtype=torch.int64))
            else:
                self.register_parameter(nm, torch.nn.Parameter(torch.zeros(e["shape"])))


SMALL_NS = [1, 2, 3, 5, 8, 9, 16, 17, 20, 24, 33]
SMALL_SHAPES = [[], [4], [7], [10], [16], [100], [432], [3456], [5120], [4097], [3, 3], [33]]


def small_manifest():
    keys = []
    for j, s in enumerate(SMALL_SHAPES):
        keys.append({"key": f"t{j}", "shape": s, "dtype": "float32"})
    keys.append({"key": "num_batches_tracked", "shape": [], "dtype": "int64"})
    keys.append({"key": "nbt_b", "shape": [], "dtype": "int64"})
    return {"name": "small", "keys": keys}


def main():
    ref = import_reference()
    torch.set_num_threads(8)
    torch.manual_seed(0)
    builders = build_models(ref)

    man_dir = os.path.join(REPO, "feddct_amd", "manifests")
    os.makedirs(man_dir, exist_ok=True)
    manifests = {}
    for name, mk in builders.items():
        m = manifest_of(name, mk())
        manifests[name] = m
        with open(os.path.join(man_dir, name + ".json"), "w") as f:
            json.dump(m, f, indent=0)
        print(name, len(m["keys"]), "keys")

    # ---- small goldens: reference server_aggregate on PRNG inputs ----------
    sm = small_manifest()
    gold = {}
    for mode in (synth.MODE_REALISTIC, synth.MODE_ADVERSARIAL):
        for n in SMALL_NS:
            for variant in ("fedavg", "fedprox"):
                g = Holder(sm)
                clients = [Holder(sm) for _ in range(n)]
                for i, c in enumerate(clients):
                    fill_module(c, sm, i, mode)
                inh = hashlib.sha256()
                for c in clients:
                    for v in c.state_dict().values():
                        inh.update(v.numpy().tobytes())
                ref[variant].server_aggregate(g, clients)
                for k, v in g.state_dict().items():
                    gold[f"{variant}/m{mode}/n{n}/{k}"] = v.numpy().copy()
                gold[f"{variant}/m{mode}/n{n}/__input_sha256"] = np.frombuffer(
                    inh.hexdigest().encode(), np.uint8)
                for c in clients:
                    for k, v in c.state_dict().items():
                        assert torch.equal(v, g.state_dict()[k]), "broadcast"
    # FedDCT / SplitFed two-model form on the small layout (main = first 6 keys)
    main_m = {"name": "small_main", "keys": sm["keys"][:6] + sm["keys"][-1:]}
    prox_m = {"name": "small_proxy", "keys": sm["keys"][6:]}
    for variant in ("feddct", "splitfed"):
        for n in (5, 24):
            gm, gp = Holder(main_m), Holder(prox_m)
            ms = [Holder(main_m) for _ in range(n)]
            ps = [Holder(prox_m) for _ in range(n)]
            for i in range(n):
                fill_module(ms[i], main_m, i, synth.MODE_ADVERSARIAL)
                fill_module(ps[i], prox_m, 100 + i, synth.MODE_ADVERSARIAL)
            ref[variant].server_aggregate(gm, gp, ms, ps)
            for k, v in gm.state_dict().items():
                gold[f"{variant}/n{n}/main/{k}"] = v.numpy().copy()
            for k, v in gp.state_dict().items():
                gold[f"{variant}/n{n}/proxy/{k}"] = v.numpy().copy()
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "small_goldens.npz"), **gold)
    with open(os.path.join(REPO, "tests", "golden", "small_manifest.json"), "w") as f:
        json.dump({"small": sm, "main": main_m, "proxy": prox_m,
                   "ns": SMALL_NS}, f, indent=0)
    print("small goldens:", len(gold), "arrays")

    # ---- full-size digests -------------------------------------------------
    digests = {}
    cases = [("fedavg", "wrn16_8_c10", 2), ("fedavg", "wrn16_8_c10", 20),
             ("fedprox", "wrn16_8_c100", 20)]
    for variant, lay, n in cases:
        g = builders[lay]()
        clients = [builders[lay]() for _ in range(n)]
        for i, c in enumerate(clients):
            fill_module(c, manifests[lay], i, synth.MODE_REALISTIC)
        ref[variant].server_aggregate(g, clients)
        d = state_digest(g)
        digests[f"{variant}/{lay}/n{n}"] = d
        print(variant, lay, n, d)
    for variant, tag, n in (("feddct", "c10", 5), ("feddct", "c100", 24)):
        lm, lp = f"wrnsl16_8_sf4_{tag}_main", f"wrnsl16_8_sf4_{tag}_proxy"
        gm, gp = builders[lm](), builders[lp]()
        ms = [builders[lm]() for _ in range(n)]
        ps = [builders[lp]() for _ in range(n)]
        for i in range(n):
            fill_module(ms[i], manifests[lm], i, synth.MODE_REALISTIC)
            fill_module(ps[i], manifests[lp], i, synth.MODE_REALISTIC)
        ref[variant].server_aggregate(gm, gp, ms, ps)
        digests[f"{variant}/{lm}/n{n}"] = state_digest(gm)
        digests[f"{variant}/{lp}/n{n}"] = state_digest(gp)
        print(variant, tag, n, digests[f"{variant}/{lm}/n{n}"], digests[f"{variant}/{lp}/n{n}"])
    digests["_meta"] = {"torch": torch.__version__, "threads": torch.get_num_threads(),
                        "cpu_capability": torch.backends.cpu.get_cpu_capability(),
                        "generator": "feddct_amd/synth.py MODE_REALISTIC, client c seed 1000+c"}
    with open(os.path.join(REPO, "tests", "golden", "digests.json"), "w") as f:
        json.dump(digests, f, indent=1)


if __name__ == "__main__":
    if sys.argv[1:] == ["--sweep"]:
        sweep_digests()
    else:
        main()
