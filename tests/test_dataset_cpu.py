"""Host side of the data path (stereo_depth_estimation_amd/dataset.py) against the reference's
behaviour: sample discovery and cache layout (dataset.py:41-83), seeded split (eval_utils.py:14-39,
pinned by tests/golden/data_path.npz), constructor validation (dataset.py:165-178), cache
require/invalid errors (dataset.py:284-295), and the augmentation factors drawn from torch's CPU
generator in the reference's order (dataset.py:214-270)."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from conftest import write_stereo_tree
from oracle import data_ref
from stereo_depth_estimation_amd import dataset as D


def test_discover_samples_layout_and_skips(tmp_path):
    write_stereo_tree(tmp_path, scenes=2, frames=3)
    (tmp_path / "not_a_scene").mkdir()  # no dataset/data: skipped
    # a frame without a right image is skipped; a .jpg left image is found
    d0 = tmp_path / "scene00" / "dataset" / "data"
    (d0 / "right/rgb/000002.png").unlink()
    (d0 / "left/rgb/000001.png").rename(d0 / "left/rgb/000001.jpg")
    s = D.discover_samples(tmp_path)
    stems = [(x.disparity_path.parent.parents[3].name, x.disparity_path.stem) for x in s]
    assert stems == [("scene00", "000000"), ("scene00", "000001"), ("scene01", "000000"), ("scene01", "000001"),
                     ("scene01", "000002")]
    assert s[1].left_rgb_path.suffix == ".jpg"
    with pytest.raises(FileNotFoundError, match="Dataset root does not exist"):
        D.discover_samples(tmp_path / "missing")


def test_cache_relpath_both_branches(tmp_path):
    write_stereo_tree(tmp_path, scenes=1, frames=1)
    s = D.discover_samples(tmp_path)[0]
    assert D.sample_cache_relpath(s).as_posix() == "scene00/000000.npz"
    odd = D.StereoSample(tmp_path / "a.png", tmp_path / "b.png", tmp_path / "d.png")
    p = D.sample_cache_relpath(odd)
    assert p.parent.name == "misc" and p.name.startswith("d_") and len(p.stem) == len("d_") + 16


def test_split_matches_reference_golden(golden_dir):
    g = np.load(golden_dir / "data_path.npz")
    for n in (10, 64):
        tr, va = D.split_samples(list(range(n)), 0.1, 42)
        assert tr == g[f"split{n}_train"].tolist() and va == g[f"split{n}_val"].tolist()
        assert (tr, va) == data_ref.split_samples(list(range(n)), 0.1, 42)
    with pytest.raises(ValueError, match="val-fraction"):
        D.split_samples([1, 2], 1.0, 0)
    with pytest.raises(ValueError, match="consumes all data"):
        D.split_samples([1], 0.5, 0)


@pytest.mark.parametrize("kw,msg", [({"blur_prob": 1.5}, "blur_prob"), ({"blur_kernel_size": 4}, "odd"),
                                    ({"blur_kernel_size": 1}, "odd"), ({"saturation_jitter": -1.0}, "saturation"),
                                    ({"gamma_jitter": -0.1}, "gamma")])
def test_constructor_validation(tmp_path, kw, msg):
    write_stereo_tree(tmp_path, scenes=1, frames=1)
    with pytest.raises(ValueError, match=msg):
        D.FoundationStereoDataset(D.discover_samples(tmp_path), **kw)
    with pytest.raises(ValueError, match="No samples"):
        D.FoundationStereoDataset([])


def test_items_are_the_decoded_uint8(tmp_path):
    ref = write_stereo_tree(tmp_path, scenes=1, frames=2)
    ds = D.FoundationStereoDataset(D.discover_samples(tmp_path), image_size=(24, 32))
    it = ds[1]
    left, right, drgb = ref["scene00/000001"]
    assert it["kind"] == 0 and it["left"].dtype == np.uint8
    assert np.array_equal(it["left"], left) and np.array_equal(it["right"], right)
    assert np.array_equal(it["disparity"], drgb)


def _reference_factor_sequence(ds):
    """The generator calls of dataset.py:214-270 for one _augment_rgb call (noise field excluded)."""
    def jit(j):
        return 1.0 if j <= 0 else float(torch.empty(1).uniform_(max(0.0, 1.0 - j), 1.0 + j).item())
    b, c, s = jit(ds.brightness_jitter), jit(ds.contrast_jitter), jit(ds.saturation_jitter)
    h = 0.0 if ds.hue_jitter <= 0 else float(torch.empty(1).uniform_(-ds.hue_jitter, ds.hue_jitter).item())
    low = max(0.1, 1.0 - ds.gamma_jitter)
    g = 1.0 if ds.gamma_jitter <= 0 else float(torch.empty(1).uniform_(low, max(low, 1.0 + ds.gamma_jitter)).item())
    blur = ds.blur_prob > 0 and ds.blur_sigma_max > 0 and bool(torch.rand(1).item() < ds.blur_prob)
    sig = float(torch.empty(1).uniform_(0.1, max(ds.blur_sigma_max, 0.1)).item()) if blur else 0.0
    n = 0.0 if ds.noise_std_max <= 0 else float(torch.empty(1).uniform_(0.0, ds.noise_std_max).item())
    return [b, c, s, h, g, sig, n]


def test_augment_factors_follow_reference_rng_order(tmp_path):
    write_stereo_tree(tmp_path, scenes=1, frames=2)
    ds = D.FoundationStereoDataset(D.discover_samples(tmp_path), augment=True, brightness_jitter=0.3,
                                   contrast_jitter=0.2, saturation_jitter=0.4, hue_jitter=0.05, gamma_jitter=0.3,
                                   blur_prob=0.5, blur_sigma_max=1.5, noise_std_max=0.0)
    torch.manual_seed(123)
    it = ds[0]
    torch.manual_seed(123)
    expect = np.array([_reference_factor_sequence(ds), _reference_factor_sequence(ds)], dtype=np.float32)
    assert it["aug"].shape == (2, 7)
    assert np.array_equal(it["aug"], expect)
    bad = D.FoundationStereoDataset(D.discover_samples(tmp_path), augment=True, hue_jitter=0.9)
    torch.manual_seed(0)
    with pytest.raises(ValueError, match="hue_factor"):
        for _ in range(8):
            bad.sample_augment_params()


def test_cache_require_and_invalid_entries(tmp_path):
    write_stereo_tree(tmp_path / "data", scenes=1, frames=1)
    samples = D.discover_samples(tmp_path / "data")
    ds = D.FoundationStereoDataset(samples, image_size=(24, 32), cache_root=tmp_path / "cache", require_cache=True)
    with pytest.raises(FileNotFoundError, match="Required cache entry"):
        ds[0]
    f = tmp_path / "cache" / D.sample_cache_relpath(samples[0])
    f.parent.mkdir(parents=True)
    np.savez(f, left=np.zeros((10, 10, 3), np.uint8), right=np.zeros((10, 10, 3), np.uint8),
             disparity=np.zeros((10, 10), np.float16))
    with pytest.raises(ValueError, match="invalid or shape-mismatched"):
        ds[0]
    lv = np.full((24, 32, 3), 7, np.uint8)
    np.savez(f, left=lv, right=lv, disparity=np.full((24, 32), 3.5, np.float16))
    it = ds[0]
    assert it["kind"] == 1 and it["disparity"].dtype == np.float16 and it["cache_file"] == ""
    # without require_cache a miss is decoded and marked for write-back
    ds2 = D.FoundationStereoDataset(samples, image_size=(24, 32), cache_root=tmp_path / "cache2")
    it2 = ds2[0]
    assert it2["kind"] == 0 and it2["cache_file"].endswith("scene00/000000.npz")


def test_collate_groups_by_kind_and_size(tmp_path):
    write_stereo_tree(tmp_path, scenes=1, frames=3)
    ds = D.FoundationStereoDataset(D.discover_samples(tmp_path), image_size=(24, 32))
    items = [ds[0], ds[1], ds[2]]
    cached = {"kind": 1, "left": np.zeros((24, 32, 3), np.uint8), "right": np.zeros((24, 32, 3), np.uint8),
              "disparity": np.zeros((24, 32), np.float16), "cache_file": ""}
    groups = D.collate_uint8([items[0], cached, items[1], items[2]])
    assert [g["kind"] for g in groups] == [0, 1]
    assert groups[0]["index"].tolist() == [0, 2, 3] and groups[1]["index"].tolist() == [1]
    assert groups[0]["left"].shape == (3, 45, 61, 3) and groups[0]["left"].dtype == torch.uint8
    assert groups[1]["disparity"].dtype == torch.int16


def test_native_cache_reader_matches_numpy_load(tmp_path):
    """sd_read_cache_batch (host C++, no GPU) returns exactly what the reference's load_cached_sample reads with
    np.load from files in its format (save_cached_sample = reference dataset.py:108-128), and rejects what the
    reference would: a missing entry, another image size. Caches written with the reference's `cache.py --compress`
    (np.savez_compressed: deflated zip members) load too, as np.load reads them."""
    rng = np.random.default_rng(3)
    H, W, n = 24, 32, 5
    paths, ref = [], []
    for i in range(n):
        left = rng.uniform(0, 1, (3, H, W)).astype(np.float32)
        right = rng.uniform(0, 1, (3, H, W)).astype(np.float32)
        tgt = rng.uniform(0, 90, (1, H, W)).astype(np.float32)
        f = tmp_path / f"s{i // 3}" / f"{i:06d}.npz"
        D.save_cached_sample(f, left, right, tgt)
        with np.load(f) as c:
            ref.append((c["left"], c["right"], c["disparity"]))
        paths.append(f)
    lt = torch.empty(n, H, W, 3, dtype=torch.uint8)
    rt = torch.empty_like(lt)
    dt = torch.empty(n, H, W, dtype=torch.int16)
    D.read_cache_batch(paths, (H, W), lt, rt, dt, threads=3)
    for i, (l_, r_, d_) in enumerate(ref):
        assert np.array_equal(lt[i].numpy(), l_) and np.array_equal(rt[i].numpy(), r_)
        assert np.array_equal(dt[i].numpy().view(np.float16), d_)
    with pytest.raises(FileNotFoundError, match="not found"):
        D.read_cache_batch(paths[:2] + [tmp_path / "missing.npz"], (H, W), lt[:3], rt[:3], dt[:3])
    with pytest.raises(ValueError, match="shape-mismatched"):
        D.read_cache_batch(paths[:1], (H, W + 8), torch.empty(1, H, W + 8, 3, dtype=torch.uint8),
                           torch.empty(1, H, W + 8, 3, dtype=torch.uint8), torch.empty(1, H, W + 8, dtype=torch.int16))
    comp = []
    for i, (l_, r_, d_) in enumerate(ref):
        comp.append(tmp_path / f"compressed{i}.npz")
        np.savez_compressed(comp[-1], left=l_, right=r_, disparity=d_)
    lt.zero_(), rt.zero_(), dt.zero_()
    D.read_cache_batch(comp[:2] + paths[2:], (H, W), lt, rt, dt, threads=2)  # mixed stored / deflated files
    for i, (l_, r_, d_) in enumerate(ref):
        assert np.array_equal(lt[i].numpy(), l_) and np.array_equal(rt[i].numpy(), r_)
        assert np.array_equal(dt[i].numpy().view(np.float16), d_)
    bad = tmp_path / "corrupt.npz"
    raw = bytearray(comp[0].read_bytes())
    raw[60:90] = bytes(30)  # clobber the first deflate stream
    bad.write_bytes(bytes(raw))
    with pytest.raises(ValueError):
        D.read_cache_batch([bad], (H, W), lt[:1], rt[:1], dt[:1])


def _png_with_filters(path, img):
    """An 8-bit RGB/RGBA PNG whose row y uses filter type y % 5 (None, Sub, Up, Average, Paeth)."""
    import struct
    import zlib

    h, w, c = img.shape
    bpp, rows, prev = c, [], np.zeros(w * c, np.int32)
    for y in range(h):
        cur = img[y].reshape(-1).astype(np.int32)
        a = np.concatenate([np.zeros(bpp, np.int32), cur[:-bpp]])
        cc = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]])
        ft = y % 5
        if ft == 0:
            pred = np.zeros_like(cur)
        elif ft == 1:
            pred = a
        elif ft == 2:
            pred = prev
        elif ft == 3:
            pred = (a + prev) // 2
        else:
            p = a + prev - cc
            pa, pb, pc = np.abs(p - a), np.abs(p - prev), np.abs(p - cc)
            pred = np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, prev, cc))
        rows.append(bytes([ft]) + ((cur - pred) % 256).astype(np.uint8).tobytes())
        prev = cur

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    ihdr = struct.pack(">IIBBBBB", w, h, 8, 2 if c == 3 else 6, 0, 0, 0)
    path.write_bytes(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(b"".join(rows)))
                     + chunk(b"IEND", b""))


def test_native_png_reader_matches_pil(tmp_path):
    """sd_read_png_batch decodes what read_rgb_uint8 (PIL convert("RGB"), reference dataset.py:184-212) returns:
    RGB and RGBA frames, every PNG row filter, PIL-written files; other kinds report False (PIL fallback)."""
    from PIL import Image

    rng = np.random.default_rng(5)
    H, W = 19, 23
    paths = []
    for i in range(6):
        img = rng.integers(0, 256, (H, W, 3 if i % 2 == 0 else 4), dtype=np.uint8)
        p = tmp_path / f"f{i}.png"
        if i < 4:
            _png_with_filters(p, img)
        else:
            Image.fromarray(img).save(p)
        paths.append(p)
    assert D.png_size(paths[0]) == (H, W)
    out = torch.empty(len(paths), H, W, 3, dtype=torch.uint8)
    assert D.read_png_batch(paths, (H, W), out, threads=3)
    for i, p in enumerate(paths):
        assert np.array_equal(out[i].numpy(), D.read_rgb_uint8(p)), i
    gray = tmp_path / "gray.png"
    Image.fromarray(rng.integers(0, 256, (H, W), dtype=np.uint8)).save(gray)
    assert not D.read_png_batch([gray], (H, W), out[:1])
    assert not D.read_png_batch(paths[:1], (H, W + 1), torch.empty(1, H, W + 1, 3, dtype=torch.uint8))
    with pytest.raises(FileNotFoundError):
        D.read_png_batch([tmp_path / "missing.png"], (H, W), out[:1])
