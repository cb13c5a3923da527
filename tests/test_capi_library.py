"""The C-ABI library: builds for gfx950, loads without a GPU, and exports every
function include/hmsc_amd.h declares (no compute calls here)."""
import ctypes
import os
import re

import numpy as np

from helpers import ROOT

HEADER = os.path.join(ROOT, "include", "hmsc_amd.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hmsc_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from hmsc_amd import build
    lib_path = build.build(verbose=False)
    lib = ctypes.CDLL(lib_path)
    names = declared_functions()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    from hmsc_amd import _lib
    assert sorted(_lib.EXPORTS) == names


def test_error_path_without_gpu_is_reported_not_raised():
    """No GPU here: device_count fails or returns 0 -- through the status code, never a crash."""
    from hmsc_amd import _lib
    L = _lib.lib()
    n = np.zeros(1, dtype=np.int32)
    rc = L.hmsc_device_count(_lib.iptr(n))
    assert rc in (0, -2)
    if rc != 0:
        assert len(L.hmsc_last_error()) > 0


def test_struct_layouts_match_header():
    """ctypes mirrors of hmsc_model / hmsc_params / hmsc_record follow the header field order."""
    from hmsc_amd import _lib
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    for struct in ("hmsc_model", "hmsc_params", "hmsc_record"):
        body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (struct, struct), text, re.S).group(1)
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            names = [re.sub(r"[\*\s]|\[.*\]", "", n) for n in decl.split(" ", 1)[1].split(",")] \
                if "," in decl else [re.sub(r"\[.*\]", "", decl.split()[-1]).lstrip("*")]
            fields.extend(names)
        ct = [f[0] for f in getattr(_lib, struct)._fields_]
        assert ct == fields, (struct, ct, fields)


def test_stale_library_is_refused(monkeypatch):
    """A library whose source stamp does not match the sources beside it is refused with a clear
    error instead of running silently (build.py writes libhmsc_amd.so.src at link time)."""
    import pytest
    from hmsc_amd import _lib, build
    build.build(verbose=False)
    monkeypatch.delenv("HMSC_AMD_LIB", raising=False)
    monkeypatch.delenv("HMSC_AMD_ALLOW_STALE", raising=False)
    _lib._check_fresh()  # the freshly built library passes
    monkeypatch.setattr(build, "source_digest", lambda: "0" * 64)
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.HmscNativeError, match="stale"):
        _lib.lib()
