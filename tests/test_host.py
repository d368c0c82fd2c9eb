"""CPU tests of the product's host side and C ABI: libpt.so loads and exports every symbol
include/pt.h declares; scene builders, OBJ loading, camera, PNG quantisation (no GPU calls)."""
import ctypes
import os
import re
import struct
import zlib

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol(pt):
    header = open(os.path.join(REPO, "include", "pt.h")).read()
    declared = set(re.findall(r"\b(pt_[a-z0-9_]+)\s*\(", header))
    assert declared == set(pt.EXPORTS), declared ^ set(pt.EXPORTS)
    lib = ctypes.CDLL(pt.LIB_PATH)
    for name in sorted(declared):
        assert hasattr(lib, name), name
    assert pt.lib.pt_abi_version() == 1


def test_library_has_gfx950_code_object(pt):
    blob = open(pt.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


@pytest.mark.parametrize("name,count", [("triangle_world", 601), ("random_world", 405), ("test_world", 3),
                                        ("rtiow", 5), ("cornell", 32), ("bunny_cornell", 5000)])
def test_presets(pt, name, count):
    p = pt.Preset(name)
    assert len(p.objects) == count
    assert (p.objects["mat"] >= 0).all() and (p.objects["mat"] < len(p.materials)).all()
    assert p.width > 0 and p.height > 0 and p.spp > 0


def test_bunny_field_size(pt):
    p = pt.Preset("bunny_field", 64, 36)
    assert len(p.objects) == 210 * 4968 + 32 == 1_043_312
    assert (p.width, p.height, p.spp, p.max_depth) == (64, 36, 512, 16)


def test_benchmark_frames(pt):
    assert (lambda p: (p.width, p.height, p.spp, p.max_depth))(pt.Preset("cornell")) == (800, 800, 256, 8)
    assert (lambda p: (p.width, p.height, p.spp, p.max_depth))(pt.Preset("bunny_cornell")) == (1920, 1080, 1024, 50)


def test_obj_loader_bunny(pt):
    tris = pt.load_obj(os.path.join(pt.MODELS_DIR, "bunny", "bunny.obj"))
    assert len(tris) == 4968
    v = tris["v"].reshape(-1, 3, 3)
    lo, hi = v.reshape(-1, 3).min(0), v.reshape(-1, 3).max(0)
    # raw bounds: x[-0.094,0.061] y[0.033,0.187] z[-0.062,0.059]
    np.testing.assert_allclose(lo, [-0.0947, 0.0330, -0.0619], atol=1e-3)
    np.testing.assert_allclose(hi, [0.0610, 0.1873, 0.0588], atol=1e-3)
    # scale + translate is v*s + t in fp32
    t2 = pt.load_obj(os.path.join(pt.MODELS_DIR, "bunny", "bunny.obj"), 2.0, (1, 2, 3), 7)
    np.testing.assert_array_equal(t2["v"].reshape(-1, 3), v.reshape(-1, 3) * np.float32(2) + np.float32([1, 2, 3]))
    assert (t2["mat"] == 7).all()


def test_obj_loader_quads_and_missing(pt, tmp_path):
    f = tmp_path / "q.obj"
    f.write_text("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvn 0 0 1\nf 1//1 2//1 3//1 4//1\n")
    t = pt.load_obj(str(f))
    assert len(t) == 2
    np.testing.assert_array_equal(t["v"][1].reshape(3, 3), [[0, 0, 0], [1, 1, 0], [0, 1, 0]])
    with pytest.raises(pt.PtError):
        pt.load_obj(str(tmp_path / "missing.obj"))


def test_bunny_cornell_placement(pt):
    p = pt.Preset("bunny_cornell")
    b = p.objects[32:]["v"].reshape(-1, 3)
    lo, hi = b.min(0), b.max(0)
    assert lo[1] > -0.1 and lo[1] < 0.1            # resting on the floor
    assert lo[0] > 290 and hi[0] < 556             # clear of the short box, inside the walls
    assert lo[2] > 0 and hi[2] < 247               # in front of the tall box


def test_camera_matches_oracle(pt, orc):
    for args in (((0, 0, 25), (0, 0, 0), 40, 16 / 9), ((278, 273, -800), (278, 273, 0), 40, 1.0),
                 ((13, 2, 3), (0, 0, 0), 20, 16 / 9), ((0, 30, 0.1), (0, 0, 0), 20, 16 / 9)):
        a = pt.camera_to_array(pt.camera_make(*args, 0.0, 10.0, 0.0, 1.0))
        b = orc.camera_make(*args, 0.0, 10.0, 0.0, 1.0)
        np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


def test_camera_move(pt):
    cam = pt.camera_make((0, 0, 25), (0, 0, 0), 40, 16 / 9)
    before = pt.camera_to_array(cam).copy()
    assert pt.lib.pt_camera_move(ctypes.byref(cam), 0, 0.4) == 0   # FORWARD: position -= front * 2.5 * dt
    after = pt.camera_to_array(cam)
    np.testing.assert_allclose(after[:3], before[:3] - np.float32([0, 0, 1]) * 1.0, atol=1e-6)
    np.testing.assert_allclose(after[3:6] - before[3:6], after[:3] - before[:3], atol=1e-5)


def test_quantize_matches_savecolor(pt):
    w, h = 5, 3
    rgb = np.linspace(-0.2, 1.3, w * h * 3, dtype=np.float32).reshape(-1, 3)
    q = pt.quantize_rgba8(rgb, w, h)
    exp = (np.clip(rgb, 0, np.float32(0.999)) * np.float32(256)).astype(np.uint8).reshape(h, w, 3)[::-1]
    np.testing.assert_array_equal(q[..., :3], exp)
    assert (q[..., 3] == 255).all()


def _read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", 0, 0
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        assert zlib.crc32(typ + body) == struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0]
        if typ == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 4 * w)
    assert (raw[:, 0] == 0).all()
    return raw[:, 1:].reshape(h, w, 4)


def test_write_png_roundtrip(pt, tmp_path):
    w, h = 7, 4
    rgb = np.random.default_rng(0).uniform(0, 1, (w * h, 3)).astype(np.float32)
    path = str(tmp_path / "x.png")
    pt.write_png(path, rgb, w, h)
    np.testing.assert_array_equal(_read_png(path), pt.quantize_rgba8(rgb, w, h))


def test_write_png_rgba8_matches_write_png(pt, orc, tmp_path):
    """A frame quantised on the device (PT_OUT_RGBA8: saveColor per pixel, rows bottom-up) and
    written with pt_write_png_rgba8 gives the same file as pt_write_png of the fp32 frame."""
    w, h = 9, 5
    rgb = np.random.default_rng(1).uniform(-0.1, 1.1, (w * h, 3)).astype(np.float32)
    a, b = str(tmp_path / "a.png"), str(tmp_path / "b.png")
    pt.write_png(a, rgb, w, h)
    pt.write_png_rgba8(b, orc.quantize_png(rgb), w, h)
    assert open(a, "rb").read() == open(b, "rb").read()


def test_quantisers_restate_reference_formulas(orc):
    c = np.float32([[-0.5, 0.0, 0.5], [0.999, 0.9995, 1.0], [1.7, 0.00390625, 0.99609375]])
    q = orc.quantize_png(c)
    np.testing.assert_array_equal(q[:, :3], [[0, 0, 128], [255, 255, 255], [255, 1, 255]])
    s = orc.quantize_surface(c)
    np.testing.assert_array_equal(s[:, :3], [[0, 0, 127], [254, 254, 255], [177, 0, 254]])
    assert (q[:, 3] == 255).all() and (s[:, 3] == 255).all()


def test_oracle_accumulate_restatement(orc):
    s1 = np.float32([[1.0, 2.0, 0.5]])
    s2 = np.float32([[3.0, 0.0, 0.25]])
    imgs = orc.accumulate([s1, s2], [2, 2])
    np.testing.assert_array_equal(imgs[0], np.sqrt(s1 * np.float32(0.5)))
    np.testing.assert_array_equal(imgs[1], np.sqrt((s1 + s2) * np.float32(0.25)))


def test_device_calls_fail_loudly_without_gpu(pt):
    if pt.device_count() > 0:
        pytest.skip("a GPU is visible")
    p = pt.Preset("cornell")
    with pytest.raises(pt.PtError) as e:
        pt.Scene(p.objects, p.materials)
    assert e.value.code == 5   # PT_ERR_NODEVICE: no CPU fallback


@pytest.mark.parametrize("name", ["cornell", "bunny_cornell", "bunny_field"])
def test_instanced_presets_flatten_to_the_flat_presets(pt, name):
    """pt_preset_instanced: meshes once in object space + translations; written out in instance
    order they are pt_preset_scene's objects bit for bit (v_world = v_object + t in float)."""
    ip, fp = pt.InstancedPreset(name), pt.Preset(name)
    parts = []
    for inst in ip.instances:
        m = inst["m"].reshape(3, 4)
        np.testing.assert_array_equal(m[:, :3], np.eye(3, dtype=np.float32))
        f, c = ip.mesh_first[inst["mesh"]], ip.mesh_count[inst["mesh"]]
        o = ip.objects[f:f + c].copy()
        o["v"] = (o["v"].reshape(-1, 3, 3) + m[:, 3]).reshape(-1, 9)
        parts.append(o)
    flat = np.concatenate(parts)
    assert ip.flattened_count() == len(fp.objects) == len(flat)
    np.testing.assert_array_equal(flat["v"], fp.objects["v"])
    np.testing.assert_array_equal(flat["mat"], fp.objects["mat"])
    np.testing.assert_array_equal(ip.materials, fp.materials)
    assert bytes(ip.camera) == bytes(fp.camera)
    if name == "bunny_field":
        assert len(ip.instances) == 211 and len(ip.objects) == 32 + 4968


def test_instanced_scene_argument_checks(pt):
    """pt_scene_create_instanced rejects bad meshes and instances before touching a device."""
    ip = pt.InstancedPreset("bunny_cornell")
    bad = ip.instances.copy()
    bad["mesh"][0] = 7
    for first, count, inst in ((ip.mesh_first, ip.mesh_count, bad),
                               (ip.mesh_first, ip.mesh_count + 1, ip.instances),
                               (ip.mesh_first, ip.mesh_count, ip.instances[:0])):
        with pytest.raises(pt.PtError) as e:
            pt.Scene.instanced(ip.objects, first, count, inst, ip.materials)
        assert e.value.code == 1   # PT_ERR_INVALID
