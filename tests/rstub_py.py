"""Python side of the stub R runtime (tests/rstub/): build R-like arguments, run a `.Call`
routine of the package's shim (src/dcor_r.c) exactly as R would, read the result back.
TEST INFRASTRUCTURE: the library is built by __graft_entry__.build()."""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "rstub", "build", "libdcor_r_stub.so")
NILSXP, LGLSXP, INTSXP, REALSXP, STRSXP, VECSXP, RAWSXP = 0, 10, 13, 14, 16, 19, 24
NA_INTEGER = -2 ** 31


class RError(RuntimeError):
    """The routine called Rf_error (R would signal an error condition)."""


class RStub:
    def __init__(self):
        import dcor  # noqa: F401  (libdcor.so first, with torch's HIP runtime)
        self.lib = C.CDLL(LIB)
        P = C.c_void_p
        for name, res, args in (("rs_nil", P, []), ("rs_real", P, [P, C.c_ssize_t]),
                                ("rs_int", P, [P, C.c_ssize_t, C.c_int]), ("rs_type", C.c_int, [P]),
                                ("rs_length", C.c_ssize_t, [P]), ("rs_nrow", C.c_int, [P]),
                                ("rs_data", P, [P]), ("rs_elt", P, [P, C.c_ssize_t]),
                                ("rs_error", C.c_char_p, []), ("rs_char", C.c_char_p, [P]),
                                ("rs_attr", P, [P, C.c_char_p]), ("rs_nargs", C.c_int, [C.c_char_p]),
                                ("rs_call", C.c_int, [C.c_char_p, C.c_int, P, P])):
            f = getattr(self.lib, name)
            f.restype, f.argtypes = res, args

    # ---- arguments
    def nil(self):
        return self.lib.rs_nil()

    def real(self, v):
        a = np.ascontiguousarray(np.atleast_1d(np.asarray(v, dtype=np.float64)))
        return self.lib.rs_real(a.ctypes.data, a.size)

    def integer(self, v):
        a = np.ascontiguousarray(np.atleast_1d(np.asarray(v, dtype=np.int32)))
        return self.lib.rs_int(a.ctypes.data, a.size, 0)

    def logical(self, v):
        a = np.ascontiguousarray(np.atleast_1d(np.asarray(v, dtype=bool)).astype(np.int32))
        return self.lib.rs_int(a.ctypes.data, a.size, 1)

    # ---- .Call
    def nargs(self, name):
        return self.lib.rs_nargs(name.encode())

    def call(self, name, *args):
        arr = (C.c_void_p * max(1, len(args)))(*args)
        out = C.c_void_p()
        rc = self.lib.rs_call(name.encode(), len(args), arr, C.byref(out))
        if rc == -1:
            raise ValueError(f"{name}: not registered with {len(args)} arguments")
        if rc == 1:
            raise RError(self.lib.rs_error().decode())
        return out.value

    def value(self, s):
        """numpy array (REAL/INTEGER/LOGICAL/RAW; matrices as [nrow, ncol]), list (VECSXP) or
        list of str (STRSXP)."""
        t, n = self.lib.rs_type(s), self.lib.rs_length(s)
        if t == VECSXP:
            return [self.value(self.lib.rs_elt(s, i)) for i in range(n)]
        if t == STRSXP:
            return [self.lib.rs_char(self.lib.rs_elt(s, i)).decode() for i in range(n)]
        if t == NILSXP:
            return None
        ct = {REALSXP: C.c_double, INTSXP: C.c_int, LGLSXP: C.c_int, RAWSXP: C.c_uint8}[t]
        if n == 0:
            return np.zeros(0, dtype=np.dtype(ct))
        a = np.ctypeslib.as_array(C.cast(self.lib.rs_data(s), C.POINTER(ct)), shape=(n,)).copy()
        nr = self.lib.rs_nrow(s)
        return a.reshape(nr, n // nr, order="F") if nr else a

    def attr(self, s, name):
        """Attribute `name` of a SEXP (as setAttrib stored it), as value() reads it; None if unset."""
        return self.value(self.lib.rs_attr(s, name.encode()))

    def type(self, s):
        return self.lib.rs_type(s)

    def elt(self, s, i):
        return self.lib.rs_elt(s, i)

    def frame(self, s):
        """A data.frame-shaped VECSXP -> (dict column -> numpy array / list, class attribute)."""
        names = self.attr(s, "names")
        return {k: self.value(self.lib.rs_elt(s, i)) for i, k in enumerate(names)}, self.attr(s, "class")
