"""GPU tests: progressive accumulation and on-device 8-bit output.

The reference's second product mode is the interactive loop (renderToGL / renderBySurface,
main.cu:307-340, 489-528) that renders a full-spp frame per display frame, with the per-pixel
streams continuing across frames, and converts to RGBA8 on the device.  Here that is
pt_render_ex with PT_OUT_RGBA8_SURFACE, plus progressive accumulation (PT_RENDER_ACCUMULATE):
every frame's linear sum is added to the film's fp32 running sums and the image is
sqrt(sum / samples so far).  The checker is the oracle's raw per-pixel sums (compat: continuing
XORWOW streams; sample mode: continuing sample indices) accumulated in float32 with numpy
(oracle.accumulate), and the saveColor / renderBySurface quantisers restated in numpy.
Bar: bit-exact.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


W, H, DEPTH = 40, 24, 50


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.fixture(scope="module")
def setup(pt, orc, gpu):
    p = pt.Preset("bunny_cornell", W, H)
    scene = pt.Scene(p.objects, p.materials, device=gpu)
    nodes = orc.build_lbvh(p.objects, orc.morton_keys(p.objects), tight=True)
    return p, scene, nodes, pt.camera_to_array(p.camera)


def test_accumulate_compat_matches_oracle(pt, orc, setup):
    p, scene, nodes, cam = setup
    film = pt.Film(W, H, seed=5)
    states = orc.film_states(5, W, film.rows)
    spps = [2, 3, 1]
    sums = []
    for spp in spps:
        _, s, _ = orc.render_sums(p.objects, p.materials, nodes, cam, W, H, film.rows, spp, DEPTH, states, nthreads=8)
        sums.append(s)
    want = orc.accumulate(sums, spps)
    for k, spp in enumerate(spps):
        rgb, st = pt.render(scene, film, p.camera, spp, DEPTH, accumulate=True)
        assert film.accumulated == sum(spps[:k + 1])
        np.testing.assert_array_equal(bits(rgb), bits(want[k]), err_msg=f"frame {k}")
    # the film's streams advanced exactly like the reference's devStates
    np.testing.assert_array_equal(film.get_rng(), states)


@pytest.mark.parametrize("kernel", ["wavefront", "simple", "wide"])
def test_accumulate_sample_matches_oracle(pt, orc, setup, kernel):
    p, scene, nodes, cam = setup
    k = {"wavefront": pt.KERNEL_WAVEFRONT, "simple": pt.KERNEL_SIMPLE, "wide": pt.KERNEL_WIDE}[kernel]
    film = pt.Film(W, H, seed=9)
    spps, chunk = [3, 5, 2], 2
    sums, base = [], 0
    for spp in spps:
        _, s, _ = orc.render_sample_sums(p.objects, p.materials, nodes, cam, W, H, film.rows, spp, DEPTH, 9, chunk,
                                         sample_base=base, nthreads=8)
        sums.append(s)
        base += spp
    want = orc.accumulate(sums, spps)
    for i, spp in enumerate(spps):
        rgb, _ = pt.render(scene, film, p.camera, spp, DEPTH, rng=pt.RNG_SAMPLE, chunk=chunk, kernel=k,
                           accumulate=True)
        np.testing.assert_array_equal(bits(rgb), bits(want[i]), err_msg=f"frame {i}")


@pytest.mark.parametrize("rng", ["compat", "sample"])
def test_first_accumulated_frame_equals_plain_frame(pt, setup, rng):
    p, scene, _, _ = setup
    r = pt.RNG_COMPAT if rng == "compat" else pt.RNG_SAMPLE
    film = pt.Film(W, H, seed=3)
    plain, _ = pt.render(scene, film, p.camera, 4, DEPTH, rng=r)
    film.reset()
    acc, _ = pt.render(scene, film, p.camera, 4, DEPTH, rng=r, accumulate=True)
    np.testing.assert_array_equal(bits(acc), bits(plain))
    # clear() restarts the accumulation: the same samples again give the same image
    film.reset()
    film.clear()
    assert film.accumulated == 0
    again, _ = pt.render(scene, film, p.camera, 4, DEPTH, rng=r, accumulate=True)
    np.testing.assert_array_equal(bits(again), bits(plain))


def test_accumulation_converges(pt, setup):
    """Progressive frames approach a high-spp reference image (error falls with samples)."""
    p, scene, _, _ = setup
    film = pt.Film(W, H, seed=11)
    ref, _ = pt.render(scene, film, p.camera, 512, DEPTH, rng=pt.RNG_SAMPLE)
    film2 = pt.Film(W, H, seed=12)
    errs = []
    for _ in range(4):
        for _ in range(4):
            rgb, _ = pt.render(scene, film2, p.camera, 4, DEPTH, rng=pt.RNG_SAMPLE, accumulate=True)
        errs.append(float(np.sqrt(np.mean((rgb ** 2 - ref ** 2) ** 2))))
    assert film2.accumulated == 64
    assert errs[-1] < errs[0] * 0.75, errs


@pytest.mark.parametrize("rng", ["compat", "sample"])
def test_rgba8_formats_match_quantisers(pt, orc, setup, rng):
    p, scene, _, _ = setup
    r = pt.RNG_COMPAT if rng == "compat" else pt.RNG_SAMPLE
    film = pt.Film(W, H, seed=2)
    rgb, _ = pt.render(scene, film, p.camera, 6, DEPTH, rng=r)
    film.reset()
    q, _ = pt.render(scene, film, p.camera, 6, DEPTH, rng=r, out_format=pt.OUT_RGBA8)
    np.testing.assert_array_equal(q, orc.quantize_png(rgb))
    film.reset()
    sfc, _ = pt.render(scene, film, p.camera, 6, DEPTH, rng=r, out_format=pt.OUT_RGBA8_SURFACE)
    np.testing.assert_array_equal(sfc, orc.quantize_surface(rgb))
    # the host quantiser (row-flipped, PngImage layout) agrees with the device one
    host = pt.quantize_rgba8(rgb, W, H).reshape(H, W, 4)[::-1].reshape(-1, 4)
    np.testing.assert_array_equal(q, host)


def test_rgba8_accumulated_device_pointer(pt, orc, setup):
    """8-bit progressive output into a device buffer (the interactive loop's surface)."""
    import torch
    p, scene, nodes, cam = setup
    film = pt.Film(W, H, seed=4)
    buf = torch.zeros(film.n_pixels * 4, dtype=torch.uint8, device="cuda:0")
    stream = torch.cuda.current_stream()
    states = orc.film_states(4, W, film.rows)
    sums = []
    for _ in range(2):
        _, s, _ = orc.render_sums(p.objects, p.materials, nodes, cam, W, H, film.rows, 3, DEPTH, states, nthreads=8)
        sums.append(s)
        pt.render(scene, film, p.camera, 3, DEPTH, out=buf.data_ptr(), stream=stream.cuda_stream, accumulate=True,
                  out_format=pt.OUT_RGBA8_SURFACE)
    torch.cuda.synchronize()
    want = orc.quantize_surface(orc.accumulate(sums, [3, 3])[-1])
    np.testing.assert_array_equal(buf.cpu().numpy().reshape(-1, 4), want)


def test_camera_move_then_clear(pt, setup):
    """processKeyboard (camera.h:41-56) then clear: the new view accumulates from zero."""
    p, scene, _, _ = setup
    cam = pt.Camera.from_buffer_copy(p.camera)
    film = pt.Film(W, H, seed=6)
    pt.render(scene, film, cam, 2, DEPTH, rng=pt.RNG_SAMPLE, accumulate=True)
    pt.camera_move(cam, 0, 0.5)
    film.clear()
    moved, _ = pt.render(scene, film, cam, 2, DEPTH, rng=pt.RNG_SAMPLE, accumulate=True)
    fresh, _ = pt.render(scene, pt.Film(W, H, seed=6), cam, 2, DEPTH, rng=pt.RNG_SAMPLE)
    np.testing.assert_array_equal(bits(moved), bits(fresh))


def test_bad_format_rejected(pt, setup):
    p, scene, _, _ = setup
    film = pt.Film(W, H, seed=1)
    with pytest.raises(pt.PtError):
        pt.render(scene, film, p.camera, 1, DEPTH, out_format=7)


@pytest.mark.parametrize("frames,rng", [(1, "compat"), (3, "sample")])
def test_render_png_app(pt, orc, gpu, tmp_path, frames, rng):
    """The C++ command-line app (main() -> renderToPng counterpart): device-quantised RGBA8
    stripes written as a PNG equal the library's frame quantised on the host."""
    import os
    import subprocess
    from helpers import read_png
    app = os.path.join(os.path.dirname(pt.LIB_PATH), "pt_render_png")
    out = str(tmp_path / "x.png")
    w, h, spp = 64, 36, 2
    r = subprocess.run([app, "--scene", "rtiow", "--models", pt.MODELS_DIR, "--width", str(w), "--height", str(h),
                        "--spp", str(spp), "--depth", "50", "--seed", "7", "--frames", str(frames), "--rng", rng,
                        "--out", out], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    p = pt.Preset("rtiow", w, h)
    scene = pt.Scene(p.objects, p.materials, device=gpu)
    film = pt.Film(w, h, seed=7)
    for _ in range(frames):
        rgb, _ = pt.render(scene, film, p.camera, spp, 50, rng=pt.RNG_COMPAT if rng == "compat" else pt.RNG_SAMPLE,
                           accumulate=frames > 1)
    np.testing.assert_array_equal(read_png(out), pt.quantize_rgba8(rgb, w, h))


@pytest.mark.parametrize("rng", ["compat", "sample"])
def test_async_frames_match_synchronous(pt, setup, rng):
    """pt_render_ex with a device output and no pt_stats returns before the frame is done
    (interactive use: camera move, clear, accumulate, display, next frame); pt_film_stats then
    waits for the film's last frame.  Queued frames give the same images and counters as the same
    frames rendered one at a time."""
    import torch
    p, scene, _, _ = setup
    r = pt.RNG_COMPAT if rng == "compat" else pt.RNG_SAMPLE
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    cams = []
    cam = pt.Camera.from_buffer_copy(bytes(p.camera))
    for k in range(4):
        pt.camera_move(cam, k % 6, 0.05)
        cams.append(pt.Camera.from_buffer_copy(bytes(cam)))

    def frames(wait):
        film = pt.Film(W, H, seed=7)
        outs, stats = [], []
        for c in cams:
            buf = torch.zeros(W * H * 4, dtype=torch.uint8, device=dev)
            film.clear(stream.cuda_stream)
            _, st = pt.render(scene, film, c, 3, DEPTH, out=buf.data_ptr(), stream=stream.cuda_stream, rng=r,
                              accumulate=True, out_format=pt.OUT_RGBA8_SURFACE, wait=wait)
            if not wait:
                assert st is None
                st = film.stats()   # waits for this frame only
            outs.append(buf)
            stats.append((st.rays, st.paths, st.node_visits))
        torch.cuda.synchronize(dev)
        return [o.cpu().numpy() for o in outs], stats

    a, sa = frames(True)
    b, sb = frames(False)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert sa == sb and all(s[1] == W * H * 3 for s in sa)


def test_film_stats_before_any_render_fails(pt, gpu):
    film = pt.Film(8, 8, seed=1, device=gpu)
    with pytest.raises(pt.PtError):
        film.stats()
