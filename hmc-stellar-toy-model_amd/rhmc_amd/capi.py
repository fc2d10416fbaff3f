"""ctypes binding of librhmc.so (include/rhmc.h).

Thin by design: argument marshalling, shape checks and error translation.
The library is REQUIRED — there is no CPU fallback; importing this module
without a built librhmc.so raises.  On a machine without a GPU the library
still loads (so its exports can be checked) but every compute entry point
returns an error.
"""
import ctypes
import os
import sys

import numpy as np

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RHMC_LIB", os.path.join(_PKG_DIR, "librhmc.so"))

RHMC_OK = 0
RHMC_ERR_ARG = -1
RHMC_ERR_HIP = -2
RHMC_ERR_NOMEM = -3
RHMC_ERR_UNSUPPORTED = -4

STATUS_NONFINITE = 1
STATUS_PLOOP_CAP = 2
STATUS_QLOOP_CAP = 4
STATUS_REFLECT_F = 8
STATUS_REFLECT_XY = 16
STATUS_NEAR_WALL = 32     # a reflection within 1e-12 of its wall

OPT_KERNEL = 1            # rhmc_ctx_set_option (include/rhmc.h)
OPT_MH_FUSED = 2
OPT_WINDOW_SPLIT = 3        # waves per chain pair in leapfrog_kr (0: by batch size)
OPT_TABLES = 4              # where WinGG keeps its factor tables (diagnostic, rhmc.h)
(TABLES_STREAM, TABLES_STREAM_POISON, TABLES_POOL, TABLES_POOL_POISON, TABLES_POOL_KEEP,
 TABLES_POOL_SYNCFREE, TABLES_POOL_BARRIER) = range(7)
# RHMC_KERNEL_* values by name
KERNELS = {"auto": 0, "generic": 1, "windowed": 2, "regwin": 3, "regwin32": 4,
           "regwin_f64": 5, "lane1": 6, "lane4": 7, "lane1_f64": 8, "pixmajor": 9,
           "multiwin": 10, "multiwin_notab": 11, "dense": 12}
# What a new Context selects unless told otherwise.  Production code leaves
# these alone; the parity tests set them (monkeypatch) to run the same inputs
# through every kernel family.  The library itself reads no environment.
DEFAULT_KERNEL = "auto"
DEFAULT_MH_FUSED = True

EXPORTS = ("rhmc_abi_version", "rhmc_device_count", "rhmc_last_error",
           "rhmc_ctx_create", "rhmc_ctx_set_image", "rhmc_ctx_image_device",
           "rhmc_ctx_destroy", "rhmc_ctx_synchronize", "rhmc_ctx_set_option",
           "rhmc_ctx_get_option", "rhmc_leapfrog",
           "rhmc_leapfrog_device", "rhmc_gradient", "rhmc_energy", "rhmc_energy_device",
           "rhmc_mh",
           "rhmc_mh_device", "rhmc_integrate", "rhmc_integrate_device",
           "rhmc_gen_image", "rhmc_gen_image_device", "rhmc_hmc_random",
           "rhmc_hmc_random_device", "rhmc_mh_scheduled", "rhmc_mh_scheduled_device",
           "rhmc_ragged_ok", "rhmc_leapfrog_ragged_device", "rhmc_energy_ragged_device",
           "rhmc_rows_copy_device", "rhmc_kinetic_rows_device")
ABI_VERSION = 4

V_FLUX_WALL = 1       # rhmc_energy f_pos bits (include/rhmc.h)
V_NO_POSCHECK = 2

SOLVER_IMPLICIT = 0
SOLVER_HMC = 1
SOLVER_RHMC_NAIVE = 2
SOLVER_RHMC_LEAPFROG = 3


class RhmcParams(ctypes.Structure):
    """Mirror of `rhmc_params` (include/rhmc.h)."""
    _fields_ = [
        ("dt", ctypes.c_double), ("delta", ctypes.c_double),
        ("B_count", ctypes.c_double), ("f_lim", ctypes.c_double),
        ("f_low", ctypes.c_double), ("fwhm_pix", ctypes.c_double),
        ("g_xx", ctypes.c_double), ("g_ff", ctypes.c_double),
        ("g_ff2", ctypes.c_double), ("g0", ctypes.c_double),
        ("g1", ctypes.c_double), ("g2", ctypes.c_double),
        ("alpha", ctypes.c_double), ("beta", ctypes.c_double),
        ("Vc_r_pow", ctypes.c_double), ("V_prior_const", ctypes.c_double),
        ("counter_max", ctypes.c_int32), ("use_prior", ctypes.c_int32),
        ("use_Vc", ctypes.c_int32), ("reserved", ctypes.c_int32),
    ]


class MhRecord(ctypes.Structure):
    """Mirror of `rhmc_mh_record` (include/rhmc.h); all fields nullable."""
    _fields_ = [("q_chain", ctypes.c_void_p), ("E_chain", ctypes.c_void_p),
                ("V_chain", ctypes.c_void_p), ("T_chain", ctypes.c_void_p),
                ("accept", ctypes.c_void_p)]


class MhSchedule(ctypes.Structure):
    """Mirror of `rhmc_mh_schedule` (include/rhmc.h): host arrays."""
    _fields_ = [("g_ff2", ctypes.c_void_p), ("beta", ctypes.c_void_p),
                ("n_g_ff2", ctypes.c_int32), ("n_beta", ctypes.c_int32)]


def make_schedule(schedule_g_ff2=None, schedule_beta=None):
    """(MhSchedule, arrays to keep alive) for run_RHMC's schedule_g_ff2 /
    schedule_beta (sampler_RHMC.py:1010-1016), or (None, ()) without one."""
    if schedule_g_ff2 is None and schedule_beta is None:
        return None, ()
    g = None if schedule_g_ff2 is None else _f64(np.ravel(schedule_g_ff2), "schedule_g_ff2")
    b = None if schedule_beta is None else _f64(np.ravel(schedule_beta), "schedule_beta")
    sc = MhSchedule(None if g is None or g.size == 0 else g.ctypes.data,
                    None if b is None or b.size == 0 else b.ctypes.data,
                    0 if g is None else g.size, 0 if b is None else b.size)
    return sc, (g, b)


class RhmcError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("librhmc error %d: %s" % (code, msg))
        self.code = code


def _load():
    if "torch" in sys.modules or os.environ.get("RHMC_IMPORT_TORCH") == "1":
        # Bind to the HIP runtime torch already loaded (same soname), so device
        # pointers and streams from torch are valid here.
        import torch  # noqa: F401
    if not os.path.exists(LIB_PATH):
        raise ImportError("librhmc.so not built at %s — run __graft_entry__.build()" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    P = ctypes.POINTER
    c_dp = P(ctypes.c_double)
    c_ip = P(ctypes.c_int32)
    vp = ctypes.c_void_p
    sig = {
        "rhmc_abi_version": (ctypes.c_int, []),
        "rhmc_device_count": (ctypes.c_int, [P(ctypes.c_int)]),
        "rhmc_last_error": (ctypes.c_char_p, []),
        "rhmc_ctx_create": (ctypes.c_int, [ctypes.c_int, c_dp, ctypes.c_int32, ctypes.c_int32, P(vp)]),
        "rhmc_ctx_set_image": (ctypes.c_int, [vp, c_dp, ctypes.c_int32, ctypes.c_int32]),
        "rhmc_ctx_image_device": (ctypes.c_int, [vp, P(vp)]),
        "rhmc_ctx_destroy": (None, [vp]),
        "rhmc_ctx_synchronize": (ctypes.c_int, [vp]),
        "rhmc_ctx_set_option": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32]),
        "rhmc_ctx_get_option": (ctypes.c_int, [vp, ctypes.c_int32, P(ctypes.c_int32)]),
        "rhmc_leapfrog": (ctypes.c_int, [vp, P(RhmcParams), c_dp, c_dp, ctypes.c_int64,
                                         ctypes.c_int32, ctypes.c_int32, c_ip, c_ip]),
        "rhmc_leapfrog_device": (ctypes.c_int, [vp, P(RhmcParams), vp, vp, ctypes.c_int64,
                                                ctypes.c_int32, ctypes.c_int32, vp, vp, vp]),
        "rhmc_gradient": (ctypes.c_int, [vp, P(RhmcParams), c_dp, c_dp, ctypes.c_int64,
                                         ctypes.c_int32, ctypes.c_int32]),
        "rhmc_energy": (ctypes.c_int, [vp, P(RhmcParams), c_dp, c_dp, c_dp, c_dp,
                                       ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
        "rhmc_energy_device": (ctypes.c_int, [vp, P(RhmcParams), vp, vp, vp, vp, ctypes.c_int64,
                                              ctypes.c_int32, ctypes.c_int32, vp]),
        "rhmc_integrate": (ctypes.c_int, [vp, P(RhmcParams), ctypes.c_int32, c_dp, c_dp,
                                          ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int32, c_ip]),
        "rhmc_integrate_device": (ctypes.c_int, [vp, P(RhmcParams), ctypes.c_int32, vp, vp,
                                                 ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                                 ctypes.c_int32, vp, vp]),
        "rhmc_mh": (ctypes.c_int, [vp, P(RhmcParams), c_dp, ctypes.c_int64, ctypes.c_int32,
                                   ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, c_dp, c_dp,
                                   ctypes.c_uint64, P(MhRecord)]),
        "rhmc_mh_device": (ctypes.c_int, [vp, P(RhmcParams), vp, ctypes.c_int64, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp,
                                          ctypes.c_uint64, P(MhRecord), vp]),
        "rhmc_mh_scheduled": (ctypes.c_int, [vp, P(RhmcParams), c_dp, ctypes.c_int64,
                                             ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_int32, c_dp, c_dp, ctypes.c_uint64,
                                             P(MhRecord), P(MhSchedule)]),
        "rhmc_mh_scheduled_device": (ctypes.c_int, [vp, P(RhmcParams), vp, ctypes.c_int64,
                                                    ctypes.c_int32, ctypes.c_int32,
                                                    ctypes.c_int32, ctypes.c_int32, vp, vp,
                                                    ctypes.c_uint64, P(MhRecord), P(MhSchedule),
                                                    vp]),
        "rhmc_hmc_random": (ctypes.c_int, [vp, P(RhmcParams), c_dp, c_dp, c_dp, c_ip,
                                           ctypes.c_int64, ctypes.c_int32, c_ip]),
        "rhmc_hmc_random_device": (ctypes.c_int, [vp, P(RhmcParams), vp, vp, vp, vp,
                                                  ctypes.c_int64, ctypes.c_int32, vp, vp]),
        "rhmc_gen_image": (ctypes.c_int, [vp, P(RhmcParams), c_dp, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, c_dp,
                                          ctypes.c_int32]),
        "rhmc_gen_image_device": (ctypes.c_int, [vp, P(RhmcParams), vp, ctypes.c_int32,
                                                 ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                 ctypes.c_uint64, vp, vp]),
        "rhmc_ragged_ok": (ctypes.c_int, [vp, P(RhmcParams), ctypes.c_int32, P(ctypes.c_int32)]),
        "rhmc_leapfrog_ragged_device": (ctypes.c_int, [vp, P(RhmcParams), vp, vp, ctypes.c_int64,
                                                       vp, vp, ctypes.c_int64, ctypes.c_int32,
                                                       ctypes.c_int32, ctypes.c_int32, vp]),
        "rhmc_energy_ragged_device": (ctypes.c_int, [vp, P(RhmcParams), vp, ctypes.c_int64, vp,
                                                     vp, ctypes.c_int64, ctypes.c_int32,
                                                     ctypes.c_int32, ctypes.c_int32, vp, vp]),
        "rhmc_rows_copy_device": (ctypes.c_int, [vp, vp, ctypes.c_int64, vp, vp, ctypes.c_int64,
                                                 vp, ctypes.c_int64, ctypes.c_int32, vp]),
        "rhmc_kinetic_rows_device": (ctypes.c_int, [vp, P(RhmcParams), vp, vp, ctypes.c_int64,
                                                    vp, vp, vp, ctypes.c_int64, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = _load()


def lib():
    return _lib


def abi_version():
    return _lib.rhmc_abi_version()


def device_count():
    n = ctypes.c_int(0)
    _lib.rhmc_device_count(ctypes.byref(n))
    return n.value


def device_available():
    return device_count() > 0


def _check(rc):
    if rc != RHMC_OK:
        raise RhmcError(rc, _lib.rhmc_last_error().decode(errors="replace"))


def _dptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _iptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def _f64(a, name):
    a = np.asarray(a)
    if a.dtype != np.float64:
        raise TypeError("%s must be float64, got %s" % (name, a.dtype))
    return np.ascontiguousarray(a)


def make_params(dt, delta, counter_max, B_count, f_lim, f_low, fwhm_pix, g_xx, g_ff,
                g_ff2, g0, g1, g2, use_prior=False, alpha=2., use_Vc=False, beta=1.,
                Vc_r_pow=1., V_prior_const=0.):
    return RhmcParams(float(dt), float(delta), float(B_count), float(f_lim), float(f_low),
                      float(fwhm_pix), float(g_xx), float(g_ff), float(g_ff2), float(g0),
                      float(g1), float(g2), float(alpha), float(beta), float(Vc_r_pow),
                      float(V_prior_const), int(counter_max), int(bool(use_prior)),
                      int(bool(use_Vc)), 0)


class Context:
    """One GPU + one data image (rhmc_ctx)."""

    def __init__(self, D, device=0, kernel=None, mh_fused=None):
        """D: the data image, or None for a context whose image comes from
        gen_image(..., install=True).  kernel: a KERNELS name (default
        DEFAULT_KERNEL), mh_fused: one-launch MH where available (default
        DEFAULT_MH_FUSED)."""
        h = ctypes.c_void_p()
        if D is None:
            _check(_lib.rhmc_ctx_create(int(device), None, 0, 0, ctypes.byref(h)))
            self.shape = None
        else:
            D = _f64(D, "D")
            if D.ndim != 2:
                raise ValueError("D must be 2-D")
            _check(_lib.rhmc_ctx_create(int(device), _dptr(D), D.shape[0], D.shape[1],
                                        ctypes.byref(h)))
            self.shape = D.shape
        self._h = h
        self.device = device
        self.set_kernel(DEFAULT_KERNEL if kernel is None else kernel)
        self.set_option(OPT_MH_FUSED, int(bool(DEFAULT_MH_FUSED if mh_fused is None
                                               else mh_fused)))

    def set_option(self, option, value):
        _check(_lib.rhmc_ctx_set_option(self._h, int(option), int(value)))

    def get_option(self, option):
        v = ctypes.c_int32()
        _check(_lib.rhmc_ctx_get_option(self._h, int(option), ctypes.byref(v)))
        return v.value

    def set_kernel(self, name):
        """Kernel family for this context's compute calls (KERNELS name)."""
        if name not in KERNELS:
            raise ValueError("unknown kernel %r (one of %s)" % (name, ", ".join(KERNELS)))
        self.set_option(OPT_KERNEL, KERNELS[name])

    @property
    def handle(self):
        return self._h

    def set_image(self, D):
        D = _f64(D, "D")
        _check(_lib.rhmc_ctx_set_image(self._h, _dptr(D), D.shape[0], D.shape[1]))
        self.shape = D.shape

    def image_device_ptr(self):
        p = ctypes.c_void_p()
        _check(_lib.rhmc_ctx_image_device(self._h, ctypes.byref(p)))
        return p.value

    def synchronize(self):
        _check(_lib.rhmc_ctx_synchronize(self._h))

    def close(self):
        if getattr(self, "_h", None):
            _lib.rhmc_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- compute ----------------------------------------------------------
    def leapfrog(self, params, q, p, n_steps, K=None, return_info=False):
        """n_steps fused RHMC_single_step()s; q, p: [n_chains, 3K] (or [3K]).
        Returns new (q, p) arrays (inputs are not mutated, like the reference)."""
        q2 = np.array(q, dtype=np.float64, order="C", copy=True)
        p2 = np.array(p, dtype=np.float64, order="C", copy=True)
        if q2.shape != p2.shape:
            raise ValueError("q and p shapes differ")
        single = q2.ndim == 1
        q2 = q2.reshape(-1, q2.shape[-1]) if not single else q2.reshape(1, -1)
        p2 = p2.reshape(q2.shape)
        if q2.shape[1] % 3:
            raise ValueError("last dimension must be 3K")
        K = q2.shape[1] // 3 if K is None else K
        n = q2.shape[0]
        it = np.zeros((n, 2), np.int32)
        st = np.zeros(n, np.int32)
        _check(_lib.rhmc_leapfrog(self._h, ctypes.byref(params), _dptr(q2), _dptr(p2), n,
                                  int(K), int(n_steps), _iptr(it), _iptr(st)))
        if single:
            q2, p2, it, st = q2[0], p2[0], it[0], st[0]
        if return_info:
            return q2, p2, it, st
        return q2, p2

    def leapfrog_device(self, params, q_ptr, p_ptr, n_chains, K, n_steps, iters_ptr=None,
                        status_ptr=None, stream=None):
        _check(_lib.rhmc_leapfrog_device(self._h, ctypes.byref(params), ctypes.c_void_p(q_ptr),
                                         ctypes.c_void_p(p_ptr), int(n_chains), int(K),
                                         int(n_steps), ctypes.c_void_p(iters_ptr or 0),
                                         ctypes.c_void_p(status_ptr or 0),
                                         ctypes.c_void_p(stream or 0)))

    def energy_device(self, params, q_ptr, p_ptr, V_ptr, T_ptr, n_chains, K, f_pos=0,
                      stream=None):
        """rhmc_energy_device: device pointers (p_ptr / T_ptr may be 0), f_pos bits."""
        _check(_lib.rhmc_energy_device(self._h, ctypes.byref(params), ctypes.c_void_p(q_ptr),
                                       ctypes.c_void_p(p_ptr or 0), ctypes.c_void_p(V_ptr or 0),
                                       ctypes.c_void_p(T_ptr or 0), int(n_chains), int(K),
                                       int(f_pos), ctypes.c_void_p(stream or 0)))

    # ---- ragged chain sets (ABI 4; device pointers, asynchronous on `stream`)
    def ragged_ok(self, params, K):
        """Whether chains of K stars can share ragged launches on this image."""
        ok = ctypes.c_int32(0)
        _check(_lib.rhmc_ragged_ok(self._h, ctypes.byref(params), int(K), ctypes.byref(ok)))
        return bool(ok.value)

    def leapfrog_ragged_device(self, params, q_ptr, p_ptr, ld, rows_ptr, K_ptr, n, K_min, K_max,
                               n_steps, stream=None):
        _check(_lib.rhmc_leapfrog_ragged_device(
            self._h, ctypes.byref(params), ctypes.c_void_p(q_ptr), ctypes.c_void_p(p_ptr),
            int(ld), ctypes.c_void_p(rows_ptr or 0), ctypes.c_void_p(K_ptr), int(n), int(K_min),
            int(K_max), int(n_steps), ctypes.c_void_p(stream or 0)))

    def energy_ragged_device(self, params, q_ptr, ld, rows_ptr, K_ptr, n, K_min, K_max, f_pos,
                             V_ptr, stream=None):
        _check(_lib.rhmc_energy_ragged_device(
            self._h, ctypes.byref(params), ctypes.c_void_p(q_ptr), int(ld),
            ctypes.c_void_p(rows_ptr or 0), ctypes.c_void_p(K_ptr), int(n), int(K_min),
            int(K_max), int(f_pos), ctypes.c_void_p(V_ptr), ctypes.c_void_p(stream or 0)))

    def rows_copy_device(self, src_ptr, ld_src, src_rows_ptr, dst_ptr, ld_dst, dst_rows_ptr, n,
                         width, stream=None):
        _check(_lib.rhmc_rows_copy_device(
            self._h, ctypes.c_void_p(src_ptr), int(ld_src), ctypes.c_void_p(src_rows_ptr or 0),
            ctypes.c_void_p(dst_ptr), int(ld_dst), ctypes.c_void_p(dst_rows_ptr or 0), int(n),
            int(width), ctypes.c_void_p(stream or 0)))

    def kinetic_rows_device(self, params, q_ptr, p_ptr, ld, K_ptr, z_ptr, zoff_ptr, n, T_ptr,
                            stream=None):
        _check(_lib.rhmc_kinetic_rows_device(
            self._h, ctypes.byref(params), ctypes.c_void_p(q_ptr), ctypes.c_void_p(p_ptr),
            int(ld), ctypes.c_void_p(K_ptr), ctypes.c_void_p(z_ptr or 0),
            ctypes.c_void_p(zoff_ptr or 0), int(n), ctypes.c_void_p(T_ptr),
            ctypes.c_void_p(stream or 0)))

    def gradient(self, params, q, kind=0):
        q2 = np.array(q, dtype=np.float64, order="C", copy=True)
        single = q2.ndim == 1
        q2 = q2.reshape(1, -1) if single else q2.reshape(-1, q2.shape[-1])
        g = np.empty_like(q2)
        _check(_lib.rhmc_gradient(self._h, ctypes.byref(params), _dptr(q2), _dptr(g),
                                  q2.shape[0], q2.shape[1] // 3, int(kind)))
        return g[0] if single else g

    def energy(self, params, q, p=None, f_pos=False, pos_check=True):
        """Returns (V, T); T is None when p is None.  pos_check=False drops the
        position support check (samplers.lightsource_gym.V has none)."""
        q2 = np.array(q, dtype=np.float64, order="C", copy=True)
        single = q2.ndim == 1
        q2 = q2.reshape(1, -1) if single else q2.reshape(-1, q2.shape[-1])
        n = q2.shape[0]
        V = np.empty(n)
        T = None
        pp = None
        if p is not None:
            pp = np.array(p, dtype=np.float64, order="C", copy=True).reshape(q2.shape)
            T = np.empty(n)
        _check(_lib.rhmc_energy(self._h, ctypes.byref(params), _dptr(q2),
                                None if pp is None else _dptr(pp), _dptr(V),
                                None if T is None else _dptr(T), n, q2.shape[1] // 3,
                                (V_FLUX_WALL if f_pos else 0) | (0 if pos_check else V_NO_POSCHECK)))
        if single:
            return V[0], (None if T is None else T[0])
        return V, T

    def mh(self, params, q, n_iter, n_steps, f_pos=True, z=None, u=None, seed=0, record=True,
           schedule_g_ff2=None, schedule_beta=None):
        """n_iter MH iterations (run_RHMC move-0 branch) of n_steps leapfrog steps
        on every chain of q [n_chains, 3K].  z [n_iter, n_chains, 3K] / u
        [n_iter, n_chains]: host randoms (None = Philox on device).
        schedule_g_ff2 / schedule_beta: run_RHMC's per-iteration schedules
        (rhmc_mh_scheduled).  Returns a dict with the final q and, when record,
        q_chain/E_chain/V_chain/T_chain [n_iter, n_chains(, 3K)] and accept
        [n_iter, n_chains]."""
        q2 = np.array(q, dtype=np.float64, order="C", copy=True)
        single = q2.ndim == 1
        q2 = q2.reshape(1, -1) if single else q2.reshape(-1, q2.shape[-1])
        n, d = q2.shape
        zz = None if z is None else _f64(z, "z").reshape(n_iter, n, d)
        uu = None if u is None else _f64(u, "u").reshape(n_iter, n)
        out = {}
        rec = None
        if record:
            out["q_chain"] = np.empty((n_iter, n, d))
            for k in ("E_chain", "V_chain", "T_chain"):
                out[k] = np.empty((n_iter, n))
            out["accept"] = np.empty((n_iter, n), np.int32)
            rec = MhRecord(out["q_chain"].ctypes.data, out["E_chain"].ctypes.data,
                           out["V_chain"].ctypes.data, out["T_chain"].ctypes.data,
                           out["accept"].ctypes.data)
        sc, keep = make_schedule(schedule_g_ff2, schedule_beta)
        _check(_lib.rhmc_mh_scheduled(
            self._h, ctypes.byref(params), _dptr(q2), n, d // 3, int(n_iter), int(n_steps),
            int(bool(f_pos)), None if zz is None else _dptr(zz),
            None if uu is None else _dptr(uu), ctypes.c_uint64(int(seed)),
            None if rec is None else ctypes.byref(rec), None if sc is None else ctypes.byref(sc)))
        del keep
        out["q"] = q2[0] if single else q2
        return out

    def mh_device(self, params, q_ptr, n_chains, K, n_iter, n_steps, f_pos=True, z_ptr=None,
                  u_ptr=None, seed=0, record=None, stream=None, schedule_g_ff2=None,
                  schedule_beta=None):
        """Device-pointer variant (asynchronous on `stream`); record: MhRecord of
        device pointers or None; schedules: host arrays (read during the call)."""
        sc, keep = make_schedule(schedule_g_ff2, schedule_beta)
        _check(_lib.rhmc_mh_scheduled_device(
            self._h, ctypes.byref(params), ctypes.c_void_p(q_ptr), int(n_chains), int(K),
            int(n_iter), int(n_steps), int(bool(f_pos)), ctypes.c_void_p(z_ptr or 0),
            ctypes.c_void_p(u_ptr or 0), ctypes.c_uint64(int(seed)),
            None if record is None else ctypes.byref(record),
            None if sc is None else ctypes.byref(sc), ctypes.c_void_p(stream or 0)))
        del keep

    def integrate(self, params, solver, q, p, n_steps, f_pos=False, return_status=False):
        """n_steps steps of integrator `solver` (SOLVER_*); returns new (q, p)."""
        q2 = np.array(q, dtype=np.float64, order="C", copy=True)
        p2 = np.array(p, dtype=np.float64, order="C", copy=True)
        single = q2.ndim == 1
        q2 = q2.reshape(1, -1) if single else q2.reshape(-1, q2.shape[-1])
        p2 = p2.reshape(q2.shape)
        st = np.zeros(q2.shape[0], np.int32)
        _check(_lib.rhmc_integrate(self._h, ctypes.byref(params), int(solver), _dptr(q2),
                                   _dptr(p2), q2.shape[0], q2.shape[1] // 3, int(n_steps),
                                   int(bool(f_pos)), _iptr(st)))
        if single:
            q2, p2, st = q2[0], p2[0], st[0]
        return (q2, p2, st) if return_status else (q2, p2)

    def hmc_random_device(self, params, dt_ptr, q_ptr, p_ptr, steps_ptr, n_chains, K,
                          status_ptr=None, stream=None):
        """Device-pointer rhmc_hmc_random (asynchronous on `stream`)."""
        _check(_lib.rhmc_hmc_random_device(self._h, ctypes.byref(params),
                                           ctypes.c_void_p(dt_ptr), ctypes.c_void_p(q_ptr),
                                           ctypes.c_void_p(p_ptr), ctypes.c_void_p(steps_ptr),
                                           int(n_chains), int(K),
                                           ctypes.c_void_p(status_ptr or 0),
                                           ctypes.c_void_p(stream or 0)))

    def integrate_device(self, params, solver, q_ptr, p_ptr, n_chains, K, n_steps, f_pos=False,
                         status_ptr=None, stream=None):
        """Device-pointer rhmc_integrate (asynchronous on `stream`)."""
        _check(_lib.rhmc_integrate_device(self._h, ctypes.byref(params), int(solver),
                                          ctypes.c_void_p(q_ptr), ctypes.c_void_p(p_ptr),
                                          int(n_chains), int(K), int(n_steps),
                                          int(bool(f_pos)), ctypes.c_void_p(status_ptr or 0),
                                          ctypes.c_void_p(stream or 0)))

    def hmc_random(self, params, dt, q, p, steps, return_status=False):
        """samplers.HMC_random trajectories (rhmc_hmc_random): per-coordinate
        step vector dt [3K], steps[c] >= 1 leapfrog steps for chain c, flux
        wall at params.f_lim.  Returns new (q, p) (p is the input momentum on
        chains whose last step flipped — the reference's stale-p quirk)."""
        q2 = np.array(q, dtype=np.float64, order="C", copy=True)
        p2 = np.array(p, dtype=np.float64, order="C", copy=True)
        single = q2.ndim == 1
        q2 = q2.reshape(1, -1) if single else q2.reshape(-1, q2.shape[-1])
        p2 = p2.reshape(q2.shape)
        K = q2.shape[1] // 3
        dt2 = np.ascontiguousarray(np.broadcast_to(np.asarray(dt, np.float64), (3 * K,)))
        st = np.zeros(q2.shape[0], np.int32)
        n = np.ascontiguousarray(np.broadcast_to(np.asarray(steps, np.int32), (q2.shape[0],)))
        _check(_lib.rhmc_hmc_random(self._h, ctypes.byref(params), _dptr(dt2), _dptr(q2),
                                    _dptr(p2), _iptr(n), q2.shape[0], K, _iptr(st)))
        if single:
            q2, p2, st = q2[0], p2[0], st[0]
        return (q2, p2, st) if return_status else (q2, p2)

    def gen_image(self, params, q, rows, cols, n_real=0, seed=0, install=False):
        """Model image (n_real=0, gen_model) or n_real Poisson realisations of it
        (gen_mock_data / gen_noise_profile) for stars q [K, 3] (flux in counts,
        x, y).  Returns [rows, cols] or [n_real, rows, cols]; install=True also
        makes image 0 this context's data image."""
        qq = np.ascontiguousarray(np.asarray(q, dtype=np.float64).reshape(-1, 3))
        K = qq.shape[0]
        out = np.empty((n_real, rows, cols) if n_real > 0 else (rows, cols))
        _check(_lib.rhmc_gen_image(self._h, ctypes.byref(params), _dptr(qq) if K else None,
                                   K, int(rows), int(cols), int(n_real),
                                   ctypes.c_uint64(int(seed)), _dptr(out), int(bool(install))))
        if install:
            self.shape = (rows, cols)
        return out

    def gen_image_device(self, params, q_ptr, K, rows, cols, n_real, seed, out_ptr, stream=None):
        _check(_lib.rhmc_gen_image_device(self._h, ctypes.byref(params),
                                          ctypes.c_void_p(q_ptr or 0), int(K), int(rows),
                                          int(cols), int(n_real), ctypes.c_uint64(int(seed)),
                                          ctypes.c_void_p(out_ptr), ctypes.c_void_p(stream or 0)))
