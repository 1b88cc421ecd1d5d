"""GPU: row-strip sharding through the C ABI, bit-exact against the unsharded frame.

In-process shards (``rc2dgi_do_group``: context k = shard k of n, distRT strips exchanged by
device copies) on one GPU, with every intermediate render texture poisoned before the frame;
each shard's colorRT / tempRT strip must equal the whole-frame result bit for bit.  The RCCL
transport is exercised at world size 1 (communicator, grouped in-place broadcast); more ranks
need more GPUs than a test box has.
"""
import numpy as np
import pytest

from conftest import rel_err  # noqa: F401  (shared helpers live there)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from radiancecascade2dglobalillumination_amd import rc2dgi

    return rc2dgi


def _scene(spec, W, H):
    from radiancecascade2dglobalillumination_amd import scenes

    if spec == "demo":
        return scenes.demo(W, H)
    if spec == "speckled":  # a random colour per occluder texel: the palettes overflow (test_gpu_parity)
        from test_gpu_parity import speckled_scene

        return speckled_scene(W, H)
    return scenes.random_scene(W, H, int(spec.split(":")[1]))


def _full(R, W, H, N, rr, rs, blur, color, emis):
    ctx = R.RC2DGI(W, H, cascade_count=N, render_scale=rs, ray_range=rr)
    ctx.set_shader_value("_BlurRadius", blur)
    ctx.frame(color, emis)
    ctx.sync()
    out = {k: ctx.download(k) for k in ("color", "temp", "dist", "jump1", "jump2", "blur", "final_gi")}
    ctx.close()
    return out


CASES = [
    # W, H, N, rayRange, renderScale, blur, world, scene
    (256, 256, 5, 3.0, 1.0, 1.5, 2, "demo"),      # fixed-tap blur + fused merge, integer JFA key
    (512, 256, 4, 2.0, 1.0, 1.5, 3, "rand:21"),   # non-square power of two: float JFA key
    (200, 120, 3, 2.0, 1.0, 2.5, 4, "rand:22"),   # non-power-of-two: float JFA taps, separate passes
    (320, 256, 4, 8.0, 0.5, 1.37, 3, "rand:23"),  # cascades coarser than the screen
    (128, 128, 3, 4.0, 1.0, 0.0, 5, "rand:24"),   # blur off
    (1024, 1024, 6, 2.0, 1.0, 1.5, 8, "demo"),
    (1200, 900, 6, 2.0, 1.0, 1.5, 8, "demo"),     # C1 size
    # strip tables (square power-of-two >= 4096: each shard builds the side tables of its own cell rows, the shards
    # exchange them and the march field; no record texture, records from the palettes or the inputs)
    (4096, 4096, 6, 2.0, 1.0, 1.5, 4, "demo"),
    (4096, 4096, 6, 2.0, 1.0, 1.5, 8, "speckled"),  # palettes overflow: records derived from colorRT / emissiveRT
    (4096, 4096, 8, 64.0, 1.0, 1.5, 2, "rand:27"),
]


@pytest.mark.parametrize("W,H,N,rr,rs,blur,world,scene", CASES)
def test_group_shards_match_whole_frame(R, W, H, N, rr, rs, blur, world, scene):
    color, emis = _scene(scene, W, H)
    want = _full(R, W, H, N, rr, rs, blur, color, emis)
    ctxs = []
    for k in range(world):
        c = R.RC2DGI(W, H, cascade_count=N, render_scale=rs, ray_range=rr)
        c.set_shader_value("_BlurRadius", blur)
        c.set_shard(k, world)
        c.set_tuning("poison", 1)
        c.upload("color", color)
        c.upload("emissive", emis)
        ctxs.append(c)
    for _ in range(2):  # the second frame checks the cross-frame ordering of the exchange
        R.do_group(ctxs)
        for c in ctxs:
            c.sync()
        for c in ctxs:
            y0, y1 = c.shard_rows()
            # the merged strip, the JumpFlood textures' own rows (computed on the strip windows with
            # the row exchange) and the whole distance field (all-gathered)
            for k in ("color", "temp", "jump1", "jump2"):
                got = c.download(k)[y0:y1]
                mism = np.count_nonzero(got != want[k][y0:y1])
                assert mism == 0, f"shard {c.shard_rows()} {k}: {mism} values differ"
            # the whole distance field (all-gathered) -- with strip tables the shards exchange the march field
            # instead, and distRT holds the own rows
            # cascadeBlurRT and the blurred final GI (cascades the size of the screen): the own rows; on the fused blur + merge
            # (power-of-two sizes) the shard holds only those (strip-sized textures)
            if c.cascade_resolution == (W, H) and blur > 0:
                for k in ("blur", "final_gi"):
                    got = c.download(k)[y0:y1]
                    mism = np.count_nonzero(got != want[k][y0:y1])
                    assert mism == 0, f"shard {c.shard_rows()} {k}: {mism} values differ"
            pow2 = (W & (W - 1)) == 0 and (H & (H - 1)) == 0
            assert c.get_tuning("blur_strip_sized") == (pow2 and c.cascade_resolution == (W, H) and 0 < blur < 3)
            st = c.get_tuning("strip_tables_active")
            assert st == (W == H and W >= 4096), (W, H, st)
            # strip tables on the fused blur + merge: giRT1 / giRT2 hold the shard's band of every direction block
            assert c.get_tuning("cascade_banded") == (st and blur > 0), (W, H, blur)
            d = c.download("dist")
            if st:
                assert np.array_equal(d[y0:y1], want["dist"][y0:y1]), f"shard {c.shard_rows()}: distRT rows"
            else:
                assert np.array_equal(d, want["dist"]), f"shard {c.shard_rows()}: distRT"
    for c in ctxs:
        c.close()


def test_shards_follow_blur_changes_between_frames(R):
    """The strip-sized blur textures (a dyadic radius on the fused blur + merge) are resized before a frame whose
    blur settings no longer take them (a non-dyadic radius, another blur path, blur off) and back: every frame's
    colorRT / final GI strips equal the unsharded frame's."""
    W = H = 256
    N, world = 4, 2
    color, emis = _scene("rand:28", W, H)
    ctxs = []
    for k in range(world):
        c = R.RC2DGI(W, H, cascade_count=N, ray_range=2.0)
        c.set_shard(k, world)
        c.set_tuning("poison", 1)
        c.upload("color", color)
        c.upload("emissive", emis)
        ctxs.append(c)
    for blur, path, sized in ((1.5, 0, 1), (1.37, 0, 0), (1.5, 2, 0), (0.0, 0, 0), (2.5, 0, 1)):
        want = _full(R, W, H, N, 2.0, 1.0, blur, color, emis)
        for c in ctxs:
            c.set_shader_value("_BlurRadius", blur)
            c.set_tuning("blur_path", path)
        R.do_group(ctxs)
        for c in ctxs:
            c.sync()
            y0, y1 = c.shard_rows()
            assert c.get_tuning("blur_strip_sized") == sized, (blur, path)
            for k in ("color", "temp") + (("final_gi",) if blur > 0 else ()):
                assert np.array_equal(c.download(k)[y0:y1], want[k][y0:y1]), (blur, path, k)
    for c in ctxs:
        c.close()


def test_sharded_context_needs_an_exchange(R):
    c = R.RC2DGI(64, 64, cascade_count=2)
    c.set_shard(1, 2)
    assert c.shard_rows() == (32, 64)
    with pytest.raises(R.RC2DGIError) as e:
        c.do_rc2dgi()
    assert e.value.code == -6
    with pytest.raises(R.RC2DGIError) as e:  # its JumpFlood exchanges rows between the steps
        c.do_phase(1)
    assert e.value.code == -6
    with pytest.raises(R.RC2DGIError):
        c.set_shard(2, 2)
    c.close()


def test_rccl_transport_single_rank(R):
    """shard_connect + do_rc2dgi with a real RCCL communicator (world 1: the grouped in-place
    broadcast runs on the context stream) -- same bits as a plain context."""
    W = H = 256
    color, emis = _scene("demo", W, H)
    want = _full(R, W, H, 4, 2.0, 1.0, 1.5, color, emis)
    c = R.RC2DGI(W, H, cascade_count=4, ray_range=2.0)
    c.set_shard(0, 1)
    c.connect(R.shard_unique_id())
    c.frame(color, emis)
    c.sync()
    assert np.array_equal(c.download("color"), want["color"])
    c.close()


def test_phase_api_matches_do(R):
    """do_phase(1) + do_phase(2) on an unsharded context is one DoRC2DGI()."""
    W, H = 192, 128
    color, emis = _scene("rand:25", W, H)
    want = _full(R, W, H, 4, 2.0, 1.0, 1.5, color, emis)
    c = R.RC2DGI(W, H, cascade_count=4, ray_range=2.0)
    c.upload("color", color)
    c.upload("emissive", emis)
    c.do_phase(1)
    ptr, pitch = c.device_buffer("dist")
    assert ptr and pitch >= W * 2
    c.do_phase(2)
    c.sync()
    assert np.array_equal(c.download("color"), want["color"])
    c.close()


@pytest.mark.parametrize("storage", ["f16", "rgba8"])
def test_group_shards_other_storage(R, storage):
    """RGBA16F cascades (RC2DGI_STORAGE_F16) and RGBA8 render textures (RC2DGI_STORAGE_RGBA8_COMPAT)
    shard the same way, bit for bit."""
    W, H, N = 512, 384, 5
    color, emis = _scene("rand:26", W, H)
    whole = R.RC2DGI(W, H, cascade_count=N, ray_range=2.0, storage=storage)
    whole.frame(color, emis)
    whole.sync()
    want = whole.download("color")
    whole.close()
    ctxs = []
    for k in range(3):
        c = R.RC2DGI(W, H, cascade_count=N, ray_range=2.0, storage=storage)
        c.set_shard(k, 3)
        c.set_tuning("poison", 1)
        c.upload("color", color)
        c.upload("emissive", emis)
        ctxs.append(c)
    R.do_group(ctxs)
    for c in ctxs:
        c.sync()
        y0, y1 = c.shard_rows()
        assert np.array_equal(c.download("color")[y0:y1], want[y0:y1])
        c.close()
