"""Checkpoint serialization from/into arenas, CPU."""
import os

import torch

from feddct_amd.arena import get_arena
from feddct_amd.checkpoint import (bucket_state_dict, load_into, save_checkpoint,
                                   save_checkpoint_main_client)
from feddct_amd.layout import BucketLayout


def net(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8),
                               torch.nn.Linear(5, 2))


def test_roundtrip_reference_format(tmp_path):
    m = net(0)
    m[1].num_batches_tracked.fill_(17)
    L = BucketLayout.from_state_dict(m.state_dict())
    get_arena(m, L)
    sd = bucket_state_dict(m)
    assert list(sd) == list(m.state_dict())
    for k, v in m.state_dict().items():
        assert torch.equal(sd[k], v) and sd[k].dtype == v.dtype
    p = save_checkpoint({"round": 3, "arch": "wide_resnet16_8", "state_dict": m,
                         "best_acc1": torch.tensor(71.5)}, True, str(tmp_path), "checkpoint_2.pth.tar")
    assert os.path.exists(tmp_path / "model_best.pth.tar")
    ck = torch.load(p, weights_only=True)
    assert ck["round"] == 3 and ck["arch"] == "wide_resnet16_8"
    # the reference's resume path: a plain module loads it unchanged
    plain = net(1)
    plain.load_state_dict(ck["state_dict"])
    for k, v in m.state_dict().items():
        assert torch.equal(plain.state_dict()[k], v)
    # and a bound module takes it with one bucket copy
    other = net(2)
    oa = get_arena(other, L)
    load_into(other, ck["state_dict"])
    assert oa.valid()
    for k, v in m.state_dict().items():
        assert torch.equal(other.state_dict()[k], v)


def test_unbound_and_feddct_helpers(tmp_path):
    m = net(3)
    sd = bucket_state_dict(m)
    assert all(torch.equal(sd[k], v) for k, v in m.state_dict().items())
    save_checkpoint_main_client({"state_dict": m.state_dict()}, False, str(tmp_path))
    assert not os.path.exists(tmp_path / "main_client_best.pth.tar")
    save_checkpoint_main_client({"state_dict": m.state_dict()}, True, str(tmp_path))
    assert os.path.exists(tmp_path / "main_client_best.pth.tar")
    other = net(4)
    load_into(other, m.state_dict())
    assert torch.equal(other[0].weight, m[0].weight)


def test_load_into_checks_slot_placement():
    """a checkpoint whose fp32 tensors share one storage of the
    bucket's size but are packed in another order must not be copied in
    bulk (that would scramble the weights); load_state_dict's path takes it."""
    m = net(5)
    L = BucketLayout.from_state_dict(m.state_dict())
    get_arena(m, L)
    want = {k: v.clone() for k, v in net(6).state_dict().items()}
    flat = torch.zeros(L.f32_numel)
    sd, off = {}, 0
    for s in reversed(L.slots):      # same total size, other placement
        if s.kind == "f32":
            flat[off:off + s.numel] = want[s.key].reshape(-1)
            sd[s.key] = flat[off:off + s.numel].view(s.shape)
            off += -(-s.numel // 64) * 64
        else:
            sd[s.key] = want[s.key]
    sd = {k: sd[k] for k in L.keys}
    assert sd[L.keys[0]].untyped_storage().nbytes() == L.f32_numel * 4
    load_into(m, sd)
    for k, v in want.items():
        assert torch.equal(m.state_dict()[k], v), k
