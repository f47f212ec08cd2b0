"""FusedAdamW against torch.optim.AdamW (the reference's optimizer, train.py:578) on the GPU.

* state_dict numbering: index i is model.parameters()[i] (registration order, enc1 first) in both
  directions, so a checkpoint's optimizer_state_dict moves between this framework and the
  reference's AdamW (train.py:421-436);
* a parameter whose .grad is None is skipped, as torch's AdamW skips it: no weight decay, no
  moment update, and its own step count starts only with its first gradient.
Tolerance: fp32 update arithmetic of the same formula in a different order, 1e-6 absolute on
parameters after a few lr=1e-3 steps.
"""

from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _models(seed=0):
    from stereo_depth_estimation_amd.model import StereoUNet

    torch.manual_seed(seed)
    hip = StereoUNet(base_channels=8, precision="fp32")
    cpu = StereoUNet(base_channels=8, precision="fp32")  # the reference's module layout, as a container
    cpu.load_state_dict(hip.state_dict())
    return hip.to(DEV), cpu


def _batch(seed=1):
    from stereo_depth_estimation_amd.data import synthetic_batch

    return synthetic_batch(2, 32, 48, seed=seed, device=DEV)


def _autograd_step(hip, opt, x, use_logvar=True):
    opt.zero_grad(set_to_none=True)
    if use_logvar:
        d, lv = hip(x, return_uncertainty=True)
        loss = (d * 0.5 + lv.exp() * 0.1).mean()
    else:
        loss = hip(x).square().mean()
    loss.backward()
    grads = {k: (None if p.grad is None else p.grad.detach().cpu().clone()) for k, p in hip.named_parameters()}
    opt.step()
    return grads


def _ref_step(cpu, ref_opt, grads):
    for k, p in cpu.named_parameters():
        p.grad = None if grads[k] is None else grads[k].clone()
    ref_opt.step()


def test_state_dict_numbering_round_trips_with_torch_adamw():
    from stereo_depth_estimation_amd.optim import FusedAdamW

    hip, cpu = _models()
    opt = FusedAdamW(hip.parameters(), lr=1e-3, weight_decay=1e-4)
    ref = torch.optim.AdamW(cpu.parameters(), lr=1e-3, weight_decay=1e-4)
    x = _batch()["input"]
    for _ in range(2):
        _ref_step(cpu, ref, _autograd_step(hip, opt, x))
    sd = opt.state_dict()
    names = [k for k, _ in cpu.named_parameters()]
    ref_sd = ref.state_dict()
    assert sorted(sd["state"]) == sorted(ref_sd["state"]) == list(range(len(names)))
    for i, k in enumerate(names):  # same index -> same parameter, same moments
        for key in ("exp_avg", "exp_avg_sq"):
            assert sd["state"][i][key].shape == ref_sd["state"][i][key].shape, (k, key)
            torch.testing.assert_close(sd["state"][i][key].cpu(), ref_sd["state"][i][key], rtol=1e-4, atol=1e-9)
        assert float(sd["state"][i]["step"]) == float(ref_sd["state"][i]["step"]) == 2.0
    # this framework's state -> the reference's AdamW, and the reference's -> FusedAdamW
    ref2 = torch.optim.AdamW(cpu.parameters(), lr=1e-3, weight_decay=1e-4)
    ref2.load_state_dict(sd)
    for i, p in enumerate(cpu.parameters()):
        assert ref2.state[p]["exp_avg"].shape == p.shape
    hip2, _ = _models()
    hip2.load_state_dict(hip.state_dict())
    opt2 = FusedAdamW(hip2.parameters(), lr=1e-3, weight_decay=1e-4)
    opt2.load_state_dict(ref_sd)
    sd2 = opt2.state_dict()
    for i, k in enumerate(names):
        torch.testing.assert_close(sd2["state"][i]["exp_avg"].cpu(), ref_sd["state"][i]["exp_avg"], rtol=0, atol=0)
        torch.testing.assert_close(sd2["state"][i]["exp_avg_sq"].cpu(), ref_sd["state"][i]["exp_avg_sq"], rtol=0,
                                   atol=0)
    # a step after loading the reference's state continues the reference's trajectory
    g = _autograd_step(hip2, opt2, x)
    _ref_step(cpu, ref, g)
    for (k, p), (_, r) in zip(hip2.named_parameters(), cpu.named_parameters()):
        torch.testing.assert_close(p.detach().cpu(), r.detach(), rtol=0, atol=1e-6, msg=k)


def test_load_rejects_mismatched_state():
    from stereo_depth_estimation_amd.optim import FusedAdamW

    hip, cpu = _models()
    opt = FusedAdamW(hip.parameters(), lr=1e-3, weight_decay=1e-4)
    ref = torch.optim.AdamW(cpu.parameters(), lr=1e-3, weight_decay=1e-4)
    x = _batch()["input"]
    _ref_step(cpu, ref, _autograd_step(hip, opt, x))
    bad = ref.state_dict()
    bad["state"] = {i: bad["state"][len(bad["state"]) - 1 - i] for i in range(len(bad["state"]))}  # reversed order
    with pytest.raises(ValueError, match="shape"):
        opt.load_state_dict(bad)


def test_grad_none_parameters_are_skipped_like_torch_adamw():
    from stereo_depth_estimation_amd.optim import FusedAdamW

    hip, cpu = _models()
    opt = FusedAdamW(hip.parameters(), lr=1e-3, weight_decay=1e-4)
    ref = torch.optim.AdamW(cpu.parameters(), lr=1e-3, weight_decay=1e-4)
    x = _batch()["input"]
    lv0 = hip.logvar_head.weight.detach().clone()
    g = _autograd_step(hip, opt, x, use_logvar=False)  # model(x): the logvar head is not in the graph
    assert g["logvar_head.weight"] is None and g["logvar_head.bias"] is None
    assert g["disparity_head.weight"] is not None
    assert torch.equal(hip.logvar_head.weight.detach(), lv0), "a grad-None parameter must not be decayed"
    _ref_step(cpu, ref, g)
    names = [k for k, _ in cpu.named_parameters()]
    sd = opt.state_dict()
    for i, k in enumerate(names):
        assert (i in sd["state"]) == (k.split(".")[0] != "logvar_head"), k
    for _ in range(2):  # then with both heads: the logvar head's own step count starts at 1
        _ref_step(cpu, ref, _autograd_step(hip, opt, x, use_logvar=True))
    for (k, p), (_, r) in zip(hip.named_parameters(), cpu.named_parameters()):
        torch.testing.assert_close(p.detach().cpu(), r.detach(), rtol=0, atol=1e-6, msg=k)
    sd, rsd = opt.state_dict(), ref.state_dict()
    for i, k in enumerate(names):
        assert float(sd["state"][i]["step"]) == float(rsd["state"][i]["step"]), k
