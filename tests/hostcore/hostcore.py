"""TEST-ONLY ctypes wrapper of libgwa_hostcore.so (kernel logic compiled for the CPU)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None


def lib():
    global _lib
    if _lib is None:
        import fcntl
        # one build at a time when several pytest-xdist workers start together
        with open(os.path.join(_HERE, ".build.lock"), "w") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            subprocess.check_call(["make", "-s", "-C", _HERE])
        L = ctypes.CDLL(os.path.join(_HERE, "libgwa_hostcore.so"))
        L.hc_index_codes.restype = ctypes.c_void_p
        L.hc_index_codes.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]
        L.hc_index_fasta.restype = ctypes.c_void_p
        L.hc_index_fasta.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
        L.hc_index_free.argtypes = [ctypes.c_void_p]
        L.hc_suspends.restype = ctypes.c_uint64
        L.hc_spec_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
        L.hc_sa.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        L.hc_align.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                               ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                               ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p]
        _lib = L
    return _lib


class HostCore:
    def __init__(self, codes=None, names=None, lengths=None, fasta=None):
        if fasta is not None:
            b = fasta.encode()
            self.h = lib().hc_index_fasta(b, len(b))
            return
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        ln = np.ascontiguousarray(lengths, dtype=np.int64)
        arr = (ctypes.c_char_p * len(names))(*[n.encode() for n in names])
        self.n = len(codes)
        self.h = lib().hc_index_codes(codes.ctypes.data, len(codes), len(names), ctypes.cast(arr, ctypes.c_void_p),
                                      ln.ctypes.data)

    def __del__(self):
        if getattr(self, "h", None):
            lib().hc_index_free(self.h)

    def sa(self, strand):
        out = np.zeros(self.n, dtype=np.uint32)
        lib().hc_sa(self.h, strand, out.ctypes.data)
        return out

    def align(self, reads, k=0.1, report_type=0, num_split=1, stats=False, strategy=0):
        n = len(reads)
        names = (ctypes.c_char_p * n)(*[r[0].encode() for r in reads])
        seqs = (ctypes.c_char_p * n)(*[r[1].encode() for r in reads])
        quals = (ctypes.c_char_p * n)(*[(r[2].encode() if r[2] is not None else None) for r in reads])
        out = ctypes.c_void_p()
        ln = ctypes.c_uint64()
        st = np.zeros(4 * n, dtype=np.int32)
        rc = lib().hc_align(self.h, k, report_type, num_split, strategy, n, ctypes.cast(names, ctypes.c_void_p),
                            ctypes.cast(seqs, ctypes.c_void_p), ctypes.cast(quals, ctypes.c_void_p), ctypes.byref(out),
                            ctypes.byref(ln), st.ctypes.data)
        if rc != 0:
            raise RuntimeError("hostcore align failed rc=%d" % rc)
        s = ctypes.string_at(out, ln.value).decode()
        return (s, st.reshape(n, 4)) if stats else s


def suspends():
    """reads the host replay of the tiers has suspended and resumed so far (all calls)"""
    return lib().hc_suspends()


def spec_stats():
    """HC_SF_COOP runs so far: (verifications run by helper lanes, passes, roll-backs)"""
    v = (ctypes.c_uint64 * 3)()
    lib().hc_spec_stats(v)
    return int(v[0]), int(v[1]), int(v[2])
