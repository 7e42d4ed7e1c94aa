"""ptrace -- Python host mirror of the hw5 render path over libpt.so (ctypes).

Mirrors the reference's in-process interface (hw5/include/scene.h:76-79):

    Scene.load(path)      <- Scene::Load(std::istream&)   (src/sceneload.cpp:112-176)
    scene.prepare()       <- Scene::InitScene()            (src/scene.cpp:7-40)
    scene.render(...)     <- Scene::Render(std::ostream&)  (src/scene.cpp:205-252)
    write_ppm(path, img)  <- the P6 write inside Render    (src/scene.cpp:206-208,243-251)

plus `Session` (tile-sharded progressive rendering on one GPU, used by bench.py
with one process per GPU).  Everything runs through the C ABI of
include/pt.h; there is no Python or CPU fallback: if libpt.so is missing the
import fails, and rendering without a gfx950 GPU raises PTError(PT_E_NO_GPU).
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PT_LIB", os.path.join(HERE, "build", "libpt.so"))

PT_OK = 0
PT_E_INVALID, PT_E_IO, PT_E_SCENE, PT_E_NO_GPU, PT_E_HIP, PT_E_RCCL, PT_E_OOM = -1, -2, -3, -4, -5, -6, -7
TRAVERSAL_REPLAY = 0
TRAVERSAL_EXACT = 1
TRAVERSAL_REPLAY_DIV = 2
GATHER_AUTO, GATHER_RCCL, GATHER_HOST = 0, 1, 2
# pt_stats.handoff sites, in PT_HO_* order (include/pt.h; PT_TUNE drop=<name>)
HANDOFF_SITES = ("suspend", "flush", "ringout", "exact", "side_take", "side_yield", "side_handon", "grow_yield",
                 "grow_handon")
ABI_VERSION = 6

# One HIP runtime per process: PyTorch bundles its own libamdhip64 (soname
# libamdhip64.so.7, but its users link the unversioned name), so loading
# libpt.so first would map the system copy and torch would then map a second
# runtime that cannot share the device.  Importing torch first makes libpt's
# DT_NEEDED libamdhip64.so.7 bind to torch's already-loaded runtime.
try:
    import torch  # noqa: F401
except ImportError:
    pass

if not os.path.exists(LIB_PATH):
    raise ImportError("libpt.so not built at %s (run `make -C raytracing-course_amd` or "
                      "`python -c 'import __graft_entry__ as g; g.build()'`)" % LIB_PATH)
_lib = C.CDLL(LIB_PATH)


class SceneInfo(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in (
        "width", "height", "samples", "ray_depth", "n_prims", "n_bvh_prims", "n_planes", "n_emitters",
        "n_nodes", "tree_depth", "max_stack", "n_aux_nodes", "aux_depth", "n_warnings")]


class RenderOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("ngpu", C.c_int32), ("spp_per_launch", C.c_uint32),
                ("samples", C.c_uint32), ("traversal", C.c_int32), ("progress", C.c_int32),
                ("win_x0", C.c_uint32), ("win_y0", C.c_uint32), ("win_w", C.c_uint32), ("win_h", C.c_uint32),
                ("gather", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("node_visits", C.c_uint64), ("prim_tests", C.c_uint64),
                ("plane_tests", C.c_uint64), ("samples", C.c_uint64), ("errors", C.c_uint64),
                ("aux_visits", C.c_uint64), ("fallbacks", C.c_uint64),
                ("kernel_ms", C.c_double), ("resolve_ms", C.c_double), ("wall_ms", C.c_double),
                ("node_bytes", C.c_uint64), ("prim_bytes", C.c_uint64), ("aux_bytes", C.c_uint64),
                ("fallbacks_ray", C.c_uint64), ("isect_ms", C.c_double), ("isect_launches", C.c_uint64),
                ("rounds", C.c_uint64), ("gather_rccl", C.c_uint64),
                ("coop_rays", C.c_uint64), ("coop_node_visits", C.c_uint64), ("coop_prim_tests", C.c_uint64),
                ("coop_aux_visits", C.c_uint64), ("coop_ms", C.c_double), ("coop_launches", C.c_uint64),
                ("short_pixels", C.c_uint64), ("handed_on", C.c_uint64), ("gather_allocs", C.c_uint64),
                ("handoff", C.c_uint64 * 12)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["handoff"] = {name: int(self.handoff[i]) for i, name in enumerate(HANDOFF_SITES)}
        return d


class SessionOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("rank", C.c_uint32), ("world", C.c_uint32), ("traversal", C.c_int32),
                ("win_x0", C.c_uint32), ("win_y0", C.c_uint32), ("win_w", C.c_uint32), ("win_h", C.c_uint32)]


_P = C.c_void_p
_sig = {
    "pt_scene_load": (C.c_int, [C.c_char_p, C.POINTER(_P)]),
    "pt_scene_load_mem": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(_P)]),
    "pt_scene_prepare": (C.c_int, [_P]),
    "pt_device_init": (C.c_int, [C.c_int]),
    "pt_gather_init": (C.c_int, [C.c_int, C.c_int]),
    "pt_scene_get_info": (C.c_int, [_P, C.POINTER(SceneInfo)]),
    "pt_scene_override": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "pt_scene_dump_bvh": (C.c_int, [_P, _P, C.c_size_t, _P, C.c_size_t]),
    "pt_scene_free": (None, [_P]),
    "pt_render_opts_default": (None, [C.POINTER(RenderOpts)]),
    "pt_render": (C.c_int, [_P, C.POINTER(RenderOpts), _P, _P, C.POINTER(Stats)]),
    "pt_write_ppm": (C.c_int, [C.c_char_p, C.c_uint32, C.c_uint32, _P]),
    "pt_session_create": (C.c_int, [_P, C.POINTER(SessionOpts), C.POINTER(_P)]),
    "pt_session_layout": (C.c_int, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
    "pt_session_trace": (C.c_int, [_P, C.c_uint32]),
    "pt_session_resolve": (C.c_int, [_P, _P, _P]),
    "pt_session_sync": (C.c_int, [_P]),
    "pt_session_reset": (C.c_int, [_P]),
    "pt_session_read_packed": (C.c_int, [_P, _P, C.c_size_t]),
    "pt_unpack_tiles": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P]),
    "pt_unpack_tiles_f32": (C.c_int, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P]),
    "pt_session_stats": (C.c_int, [_P, C.POINTER(Stats)]),
    "pt_session_stream": (_P, [_P]),
    "pt_session_free": (None, [_P]),
    "pt_last_error": (C.c_char_p, []),
    "pt_abi_version": (C.c_int, []),
    "pt_selftest_ray_intersection": (C.c_int, [_P, C.c_int32, C.c_uint32, _P, _P, _P, _P]),
    "pt_selftest_render_host": (C.c_int, [_P, C.c_int32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                          C.c_uint32, _P]),
    "pt_selftest_gamma_table": (C.c_int, [_P, _P]),
}
for _name, (_res, _args) in _sig.items():
    _f = getattr(_lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = tuple(_sig)


class PTError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (code %d)" % (msg, code))
        self.code = code


def _check(rc):
    if rc != PT_OK:
        raise PTError(rc, _lib.pt_last_error().decode(errors="replace"))
    return rc


def last_error():
    """pt_last_error(): the message of the calling thread's last failure (also one a call
    recovered from, such as the RCCL gather's fail-over to the host)."""
    return _lib.pt_last_error().decode(errors="replace")


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


class Scene:
    """A loaded hw5 scene (owns the native pt_scene)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def load(cls, path):
        h = _P()
        _check(_lib.pt_scene_load(os.fsencode(path), C.byref(h)))
        return cls(h)

    @classmethod
    def loads(cls, text):
        b = text.encode() if isinstance(text, str) else bytes(text)
        h = _P()
        _check(_lib.pt_scene_load_mem(b, len(b), C.byref(h)))
        return cls(h)

    def close(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.pt_scene_free(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def prepare(self):
        _check(_lib.pt_scene_prepare(self._h))
        return self

    def override(self, width=0, height=0, samples=0, ray_depth=0):
        _check(_lib.pt_scene_override(self._h, width, height, samples, ray_depth))
        return self

    @property
    def info(self):
        i = SceneInfo()
        _check(_lib.pt_scene_get_info(self._h, C.byref(i)))
        return {k: getattr(i, k) for k, _ in i._fields_}

    def dump_bvh(self):
        """(nodes bytes, prims bytes) in the SURVEY §8c fingerprint layout."""
        inf = self.info
        nb = np.zeros(inf["n_nodes"] * 40, np.uint8)
        pb = np.zeros(inf["n_prims"] * 52, np.uint8)
        _check(_lib.pt_scene_dump_bvh(self._h, _ptr(nb), nb.nbytes, _ptr(pb), pb.nbytes))
        return nb.tobytes(), pb.tobytes()

    def render(self, device=0, ngpu=1, samples=0, spp_per_launch=0, radiance=False, progress=False, window=None,
               traversal=TRAVERSAL_REPLAY, gather=GATHER_AUTO):
        """Render on the GPU(s): returns (rgb u8 HxWx3, radiance f32 HxWx3 | None, stats).

        window=(x0, y0, w, h) renders only those pixels (global-index seeds kept).
        gather: GATHER_AUTO (RCCL when ngpu > 1), GATHER_RCCL (RCCL at any ngpu, an
        error if it fails), GATHER_HOST (never RCCL)."""
        inf = self.info
        w, h = (window[2], window[3]) if window else (inf["width"], inf["height"])
        rgb = np.zeros((h, w, 3), np.uint8)
        rad = np.zeros((h, w, 3), np.float32) if radiance else None
        o = RenderOpts()
        _lib.pt_render_opts_default(C.byref(o))
        o.device, o.ngpu, o.samples, o.spp_per_launch, o.progress = device, ngpu, samples, spp_per_launch, int(progress)
        o.traversal = traversal
        o.gather = gather
        if window:
            o.win_x0, o.win_y0, o.win_w, o.win_h = window
        st = Stats()
        _check(_lib.pt_render(self._h, C.byref(o), _ptr(rgb), _ptr(rad), C.byref(st)))
        return rgb, rad, st.as_dict()

    # test hooks (host execution of the device traversal code; not a render path)
    def selftest_ray_intersection(self, rays, traversal=TRAVERSAL_REPLAY):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
        ids = np.zeros(len(rays), np.int32)
        hits = np.zeros((len(rays), 5), np.float32)
        ctr = np.zeros(8, np.uint64)
        _check(_lib.pt_selftest_ray_intersection(self._h, traversal, len(rays), _ptr(rays), _ptr(ids), _ptr(hits),
                                                 _ptr(ctr)))
        return ids, hits, {"nodes": int(ctr[1]), "prim_tests": int(ctr[2]), "aux": int(ctr[5]),
                           "fallbacks": int(ctr[6])}

    def selftest_render_host(self, x0, y0, w, h, spp=0, traversal=TRAVERSAL_REPLAY):
        rad = np.zeros((h, w, 3), np.float32)
        _check(_lib.pt_selftest_render_host(self._h, traversal, x0, y0, w, h, spp, _ptr(rad)))
        return rad

    def gamma_table(self):
        t = np.zeros(256, np.float32)
        _check(_lib.pt_selftest_gamma_table(self._h, _ptr(t)))
        return t


class Session:
    """Tile-sharded progressive renderer on one device (include/pt.h sessions)."""

    def __init__(self, scene, device=0, rank=0, world=1, traversal=TRAVERSAL_REPLAY, window=None):
        self.scene = scene
        o = SessionOpts(device, rank, world, traversal, *(window or (0, 0, 0, 0)))
        self._h = _P()
        _check(_lib.pt_session_create(scene._h, C.byref(o), C.byref(self._h)))
        nt, nb = C.c_uint32(), C.c_uint64()
        _check(_lib.pt_session_layout(self._h, C.byref(nt), C.byref(nb)))
        self.n_tiles, self.packed_bytes = nt.value, nb.value
        self.rank, self.world = rank, world

    def trace(self, spp):
        _check(_lib.pt_session_trace(self._h, spp))

    def resolve(self, dev_out=None, dev_rad=None):
        _check(_lib.pt_session_resolve(self._h, dev_out, dev_rad))

    def sync(self):
        _check(_lib.pt_session_sync(self._h))

    def reset(self):
        """Restart every owned pixel at sample 0 (buffers and counters kept): the next
        trace(S) renders what a new session would."""
        _check(_lib.pt_session_reset(self._h))

    def read_packed(self):
        out = np.zeros(self.packed_bytes, np.uint8)
        _check(_lib.pt_session_read_packed(self._h, _ptr(out), out.nbytes))
        return out

    def stats(self):
        st = Stats()
        _check(_lib.pt_session_stats(self._h, C.byref(st)))
        return st.as_dict()

    @property
    def stream(self):
        return _lib.pt_session_stream(self._h)

    def close(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.pt_session_free(self._h)
            self._h = None

    __del__ = close


def tile_owner(t, tiles_x, world):
    """the rank that owns window tile t (include/pt.h sessions; pt_kernels.h tile_owner)"""
    return (t % tiles_x + t // tiles_x) % world


def rank_tiles(width, height, rank, world):
    """the window tiles of `rank`, in its local (ascending) order"""
    tiles_x, tiles_y = (width + 15) // 16, (height + 15) // 16
    return [t for t in range(tiles_x * tiles_y) if tile_owner(t, tiles_x, world) == rank]


def unpack_tiles(packed, width, height, rank, world, out=None):
    out = np.zeros((height, width, 3), np.uint8) if out is None else out
    packed = np.ascontiguousarray(packed, np.uint8)
    _check(_lib.pt_unpack_tiles(width, height, rank, world, _ptr(packed), _ptr(out)))
    return out


def unpack_tiles_f32(packed, width, height, rank, world, out=None):
    out = np.zeros((height, width, 3), np.float32) if out is None else out
    packed = np.ascontiguousarray(packed, np.float32)
    _check(_lib.pt_unpack_tiles_f32(width, height, rank, world, _ptr(packed), _ptr(out)))
    return out


def write_ppm(path, rgb):
    rgb = np.ascontiguousarray(rgb, np.uint8)
    h, w, _ = rgb.shape
    _check(_lib.pt_write_ppm(os.fsencode(path), w, h, _ptr(rgb)))


def abi_version():
    return _lib.pt_abi_version()
