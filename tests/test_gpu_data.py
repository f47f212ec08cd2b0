"""On-device data path (csrc/data.hip via stereo_depth_estimation_amd/dataset.py).

* sd_stereo_preprocess against items the REFERENCE's FoundationStereoDataset produced from PNG
  files (tests/golden/data_path.npz, gen_golden.py) and against the numpy restatement
  (oracle/data_ref.py) at a realistic downscale. Tolerance: 2e-6 absolute on the [0,1] RGB
  channels and 1e-6 relative on disparity (fp32 re-association of the bilinear sum only; the
  decode is exact), the valid mask exact.
* sd_stereo_from_cache against load_cached_sample (dataset.py:86-105): exact.
* sd_augment_rgb against the torchvision-0.25 restatement (oracle/aug_ref.py; parity unpinned by
  the reference) with the noise off: 2e-5 absolute (powf/expf ulps, HSV round trip).
  With noise on: the added field has mean 0 and the requested std (statistical).
* DeviceLoader end to end on a PNG tree, including the cache round trip (write on miss in the
  reference's format, read back as cached samples).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import write_stereo_tree
from oracle import aug_ref, data_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def L():
    from stereo_depth_estimation_amd import _lib

    _lib.load()
    return _lib


def _prep(lib, left, right, drgb, out_hw):
    B, Hs, Ws, _ = left.shape
    Ho, Wo = out_hw
    l_d, r_d, d_d = (torch.from_numpy(np.ascontiguousarray(a)).to(DEV) for a in (left, right, drgb))
    inp = torch.empty(B, 6, Ho, Wo, device=DEV)
    tgt = torch.empty(B, 1, Ho, Wo, device=DEV)
    val = torch.empty(B, 1, Ho, Wo, device=DEV, dtype=torch.bool)
    lib.call("sd_stereo_preprocess", l_d.data_ptr(), r_d.data_ptr(), d_d.data_ptr(), B, Hs, Ws, Ho, Wo, inp.data_ptr(),
             tgt.data_ptr(), val.data_ptr(), lib.stream_handle())
    torch.cuda.synchronize()
    return inp.cpu().numpy(), tgt.cpu().numpy(), val.cpu().numpy()


def test_preprocess_matches_reference_dataset_items(golden_dir):
    lib = L()
    g = np.load(golden_dir / "data_path.npz")
    left = np.stack([g[f"src{i}_left"] for i in range(4)])
    right = np.stack([g[f"src{i}_right"] for i in range(4)])
    drgb = np.stack([g[f"src{i}_disp_rgb"] for i in range(4)])
    inp, tgt, val = _prep(lib, left, right, drgb, (24, 32))
    for i in range(4):
        assert np.abs(inp[i] - g[f"item{i}_input"]).max() <= 2e-6
        rt = g[f"item{i}_target"]
        assert np.abs(tgt[i] - rt).max() <= 1e-6 * (1 + np.abs(rt).max())
        assert np.array_equal(val[i], g[f"item{i}_valid"])


@pytest.mark.parametrize("src_hw,out_hw", [((480, 640), (240, 320)), ((375, 1242), (240, 320)), ((17, 23), (40, 50))])
def test_preprocess_matches_restatement(src_hw, out_hw):
    lib = L()
    rng = np.random.default_rng(7)
    B = 2
    left = rng.integers(0, 256, (B, *src_hw, 3), dtype=np.uint8)
    right = rng.integers(0, 256, (B, *src_hw, 3), dtype=np.uint8)
    disp = rng.uniform(0, 200, (B, *src_hw)).astype(np.float32)
    disp[rng.random((B, *src_hw)) < 0.1] = 0
    drgb = data_ref.encode_disparity_to_rgb(disp)
    inp, tgt, val = _prep(lib, left, right, drgb, out_hw)
    for b in range(B):
        ref_in = np.concatenate([data_ref.load_rgb_from_uint8(left[b], out_hw),
                                 data_ref.load_rgb_from_uint8(right[b], out_hw)])
        ref_t = data_ref.load_disparity_from_rgb24(drgb[b], out_hw)
        assert np.abs(inp[b] - ref_in).max() <= 2e-6
        assert np.abs(tgt[b] - ref_t).max() <= 1e-6 * (1 + np.abs(ref_t).max())
        assert np.array_equal(val[b], ref_t > 0)


def test_from_cache_matches_load_cached_sample():
    lib = L()
    rng = np.random.default_rng(3)
    B, H, W = 3, 24, 32
    left = rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)
    right = rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)
    disp = rng.uniform(-1, 50, (B, H, W)).astype(np.float16)
    l_d, r_d = torch.from_numpy(left).to(DEV), torch.from_numpy(right).to(DEV)
    d_d = torch.from_numpy(disp).to(DEV).view(torch.int16)
    inp = torch.empty(B, 6, H, W, device=DEV)
    tgt = torch.empty(B, 1, H, W, device=DEV)
    val = torch.empty(B, 1, H, W, device=DEV, dtype=torch.bool)
    lib.call("sd_stereo_from_cache", l_d.data_ptr(), r_d.data_ptr(), d_d.data_ptr(), B, H, W, inp.data_ptr(),
             tgt.data_ptr(), val.data_ptr(), lib.stream_handle())
    torch.cuda.synchronize()
    for b in range(B):
        ref_l = torch.from_numpy(left[b].astype(np.float32) / 255.0).permute(2, 0, 1)
        ref_r = torch.from_numpy(right[b].astype(np.float32) / 255.0).permute(2, 0, 1)
        ref_t = torch.from_numpy(disp[b].astype(np.float32)).unsqueeze(0)
        assert torch.equal(inp[b].cpu(), torch.cat([ref_l, ref_r]))
        assert torch.equal(tgt[b].cpu(), ref_t)
        assert torch.equal(val[b].cpu(), ref_t > 0)


def _augment(lib, x, params, ks, seed=1):
    B, _, H, W = x.shape
    xd = x.clone().to(DEV)
    pd = torch.tensor(params, dtype=torch.float32).reshape(2 * B, 7).to(DEV)
    work = torch.empty(B * 6 * H * W + 128 * B, device=DEV)
    lib.call("sd_augment_rgb", xd.data_ptr(), B, H, W, pd.data_ptr(), ks, seed, work.data_ptr(), lib.stream_handle())
    torch.cuda.synchronize()
    return xd.cpu()


def test_augment_matches_torchvision_restatement():
    lib = L()
    torch.manual_seed(0)
    B, H, W, ks = 3, 37, 53, 5
    x = torch.rand(B, 6, H, W)
    x[0, :, :4, :4] = 0.5  # grey patch: hue of equal channels
    params = []
    for im in range(2 * B):
        sigma = [0.0, 0.7, 1.9][im % 3]
        params.append([0.7 + 0.1 * im, 1.3 - 0.1 * im, 0.6 + 0.15 * im, [-0.08, 0.0, 0.05][im % 3], 0.8 + 0.07 * im,
                       sigma, 0.0])
    got = _augment(lib, x, params, ks)
    for im in range(2 * B):
        b, side = im // 2, im % 2
        img = x[b, side * 3:side * 3 + 3]
        p = params[im]
        ref = aug_ref.augment_rgb(img.clone(), p[0], p[1], p[2], p[3], p[4], p[5], ks)
        assert float((got[b, side * 3:side * 3 + 3] - ref).abs().max()) <= 2e-5, f"image {im}"


def test_augment_noise_statistics_and_clamp():
    lib = L()
    B, H, W = 2, 128, 160
    x = torch.full((B, 6, H, W), 0.5)
    std = 0.05
    params = [[1.0, 1.0, 1.0, 0.0, 1.0, 0.0, std]] * (2 * B)
    got = _augment(lib, x, params, 5, seed=11)
    d = (got - 0.5).flatten()
    assert abs(float(d.mean())) < 1e-3
    assert abs(float(d.std()) - std) < 1e-3
    again = _augment(lib, x, params, 5, seed=11)
    assert torch.equal(got, again)  # deterministic for a seed
    big = _augment(lib, x, [[1.0, 1.0, 1.0, 0.0, 1.0, 0.0, 2.0]] * (2 * B), 5, seed=5)
    assert float(big.min()) >= 0.0 and float(big.max()) <= 1.0


def test_device_loader_end_to_end_with_cache(tmp_path):
    from stereo_depth_estimation_amd import dataset as D

    ref = write_stereo_tree(tmp_path / "data", scenes=2, frames=3, hw=(45, 61), seed=2)
    samples = D.discover_samples(tmp_path / "data")
    ds = D.FoundationStereoDataset(samples, image_size=(24, 32), cache_root=tmp_path / "cache")
    loader = D.DeviceLoader(ds, batch_size=4, shuffle=False, num_workers=0, device=DEV)
    batches = list(loader)
    assert [b["input"].shape[0] for b in batches] == [4, 2]
    torch.cuda.synchronize()
    keys = sorted(ref)
    allin = torch.cat([b["input"] for b in batches]).cpu().numpy()
    allt = torch.cat([b["target"] for b in batches]).cpu().numpy()
    allv = torch.cat([b["valid_mask"] for b in batches]).cpu().numpy()
    for i, k in enumerate(keys):
        left, right, drgb = ref[k]
        ref_in = np.concatenate([data_ref.load_rgb_from_uint8(left, (24, 32)), data_ref.load_rgb_from_uint8(right, (24, 32))])
        ref_t = data_ref.load_disparity_from_rgb24(drgb, (24, 32))
        assert np.abs(allin[i] - ref_in).max() <= 2e-6
        assert np.abs(allt[i] - ref_t).max() <= 1e-6 * (1 + np.abs(ref_t).max())
        assert np.array_equal(allv[i], ref_t > 0)
    # the first pass wrote the reference's cache files; a second pass reads them (uint8 RGB, f16 disparity)
    files = sorted((tmp_path / "cache").rglob("*.npz"))
    assert len(files) == 6
    with np.load(files[0]) as c:
        assert c["left"].dtype == np.uint8 and c["left"].shape == (24, 32, 3) and c["disparity"].dtype == np.float16
    ds2 = D.FoundationStereoDataset(samples, image_size=(24, 32), cache_root=tmp_path / "cache", require_cache=True)
    b2 = torch.cat([b["input"] for b in D.DeviceLoader(ds2, batch_size=6, device=DEV)]).cpu().numpy()
    assert np.abs(b2 - np.round(allin * 255).clip(0, 255) / 255).max() <= 1 / 255 + 1e-6


def test_run_epoch_on_device_loader(tmp_path):
    from stereo_depth_estimation_amd import dataset as D
    from stereo_depth_estimation_amd.model import StereoUNet
    from stereo_depth_estimation_amd.optim import FusedAdamW
    from stereo_depth_estimation_amd.train import run_epoch

    write_stereo_tree(tmp_path, scenes=1, frames=4, hw=(40, 52), seed=4)
    ds = D.FoundationStereoDataset(D.discover_samples(tmp_path), image_size=(32, 48), augment=True,
                                   brightness_jitter=0.2, hue_jitter=0.05, blur_prob=0.5, blur_sigma_max=1.0,
                                   noise_std_max=0.02)
    torch.manual_seed(0)
    model = StereoUNet(in_channels=6, out_channels=1, base_channels=8).to(DEV)
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
    metrics, step = run_epoch(model, D.DeviceLoader(ds, batch_size=2, shuffle=True, device=DEV), DEV, optimizer=opt)
    assert step == 2 and set(metrics) == {"loss", "nll", "mae", "rmse", "sigma"}
    assert all(np.isfinite(v) for v in metrics.values())


def test_device_loader_native_reader_matches_dataloader_path(tmp_path):
    """DeviceLoader(native=True) (in-process C++ cache reader, two pinned buffer sets) yields the same batches, in
    the same shuffled order, as the DataLoader worker path over the same cache; it is the default for a
    require_cache dataset without augmentation."""
    from stereo_depth_estimation_amd import dataset as D

    write_stereo_tree(tmp_path / "data", scenes=2, frames=5, hw=(45, 61), seed=7)
    samples = D.discover_samples(tmp_path / "data")
    ds = D.FoundationStereoDataset(samples, image_size=(24, 32), cache_root=tmp_path / "cache")
    for _ in D.DeviceLoader(ds, batch_size=4, device=DEV):  # first pass writes the cache
        pass
    torch.cuda.synchronize()
    dsc = D.FoundationStereoDataset(samples, image_size=(24, 32), cache_root=tmp_path / "cache", require_cache=True)
    assert D.DeviceLoader(dsc, batch_size=3, device=DEV).native
    runs = {}
    for native in (True, False):
        ld = D.DeviceLoader(dsc, batch_size=3, shuffle=True, device=DEV, generator=torch.Generator().manual_seed(5),
                            native=native, num_workers=0 if native else 2)
        assert ld.native is native
        runs[native] = [{k: v.cpu() for k, v in b.items()} for b in ld]
    assert [b["input"].shape[0] for b in runs[True]] == [3, 3, 3, 1]
    for a, b in zip(runs[True], runs[False]):
        for k in ("input", "target", "valid_mask"):
            assert torch.equal(a[k], b[k]), k
    # with augmentation: the factors and noise seeds come from the global RNG in a num_workers=0 DataLoader's order
    dsa = D.FoundationStereoDataset(samples, image_size=(24, 32), cache_root=tmp_path / "cache", require_cache=True,
                                    augment=True, brightness_jitter=0.2, hue_jitter=0.05, blur_prob=0.5,
                                    blur_sigma_max=1.0, noise_std_max=0.02)
    runs = {}
    for native in (True, False):
        torch.manual_seed(11)
        ld = D.DeviceLoader(dsa, batch_size=4, shuffle=True, device=DEV, native=native, num_workers=0)
        runs[native] = [{k: v.cpu() for k, v in b.items()} for _ in range(2) for b in ld]  # two epochs
    assert len(runs[True]) == len(runs[False]) == 6
    for a, b in zip(runs[True], runs[False]):
        for k in ("input", "target", "valid_mask"):
            assert torch.equal(a[k], b[k]), ("aug", k)


def test_device_loader_native_png_matches_dataloader_path(tmp_path):
    """DeviceLoader(native=True) on an un-cached PNG dataset (frames decoded by the C++ reader, then the same
    sd_stereo_preprocess) equals the DataLoader path, plain and with augmentation (RNG in a num_workers=0 order)."""
    from stereo_depth_estimation_amd import dataset as D

    write_stereo_tree(tmp_path / "data", scenes=2, frames=5, hw=(45, 61), seed=9)
    samples = D.discover_samples(tmp_path / "data")
    for aug in (False, True):
        ds = D.FoundationStereoDataset(samples, image_size=(24, 32), augment=aug, brightness_jitter=0.2,
                                       hue_jitter=0.05, blur_prob=0.5, blur_sigma_max=1.0, noise_std_max=0.02)
        assert not D.DeviceLoader(ds, batch_size=3, device=DEV).native  # opt-in for PNG sources
        runs = {}
        for native in (True, False):
            torch.manual_seed(13)
            ld = D.DeviceLoader(ds, batch_size=3, shuffle=True, device=DEV, native=native, num_workers=0)
            runs[native] = [{k: v.cpu() for k, v in b.items()} for b in ld]
        assert [b["input"].shape[0] for b in runs[True]] == [3, 3, 3, 1]
        for a, b in zip(runs[True], runs[False]):
            for k in ("input", "target", "valid_mask"):
                assert torch.equal(a[k], b[k]), (aug, k)
