"""CPU-side checks of the C ABI: the library loads, exports every symbol the
header declares, its host statistics match the reference KATs, and compute
entry points fail loudly (no CPU fallback) when no GPU is visible."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import engine_bind as eb

gs = eb.gs
ROOT = eb.ROOT
HEADER = os.path.join(ROOT, "include", "gossip_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gs_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    lib = C.CDLL(gs.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert missing == []
    # and the Python binding wraps every one of them
    assert set(syms) <= set(gs.EXPORTS)


def test_no_cpu_fallback_without_gpu():
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import engine_bind as eb; import numpy as np\n"
            "try:\n    eb.gs.Engine(np.arange(1, 20, dtype=np.uint64) * 10**9, 1)\n"
            "except eb.gs.GsError as e:\n    print('RAISED', e.code)\n" % os.path.join(ROOT, "tests"))
    env = dict(os.environ, HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="-1")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert "RAISED" in out.stdout, out.stdout + out.stderr


def test_hops_stat_kat():
    # gossip_stats.rs:2159-2259 through the product's host statistics
    M = 2**64 - 1
    assert gs.hops_stat([M, M, M, M, 0, 1, 1, 2, 2, 3]) == (1.8, 2.0, 3, 1)
    assert gs.hops_stat([M, M, M, M, M, M, 0, 1, 1, 2]) == (1.3333333333333333, 1.0, 2, 1)
    assert gs.hops_stat([M, M, M, M, M, M, M, 0, 1, 6]) == (3.5, 3.5, 6, 1)
    # aggregate over the raw collection (0s kept, filtered by HopsStat)
    raw = [0, 1, 1, 2, 2, 3, 0, 1, 1, 2, 0, 1, 6]
    assert gs.hops_stat(raw) == (2.0, 1.5, 6, 1)
    assert gs.hops_stat([3, 2, 6]) == (3.6666666666666665, 3.0, 6, 2)


def test_stat_collection_kat():
    # gossip_stats.rs:2261-2359
    assert gs.stat_collection([0.6]) == (0.6, 0.6, 0.6, 0.6)
    assert gs.stat_collection([0.6, 0.4]) == (0.5, 0.5, 0.6, 0.4)
    assert gs.stat_collection([0.6, 0.4, 0.2]) == (0.4000000000000001, 0.4, 0.6, 0.2)


def test_ids_follow_base58_order():
    pks = [i.to_bytes(8, "big") + bytes(24) for i in range(1, 7)]
    # counters 1 and 2 encode to shorter strings that sort after 3..6
    assert gs.ids_from_pubkeys(pks) == [4, 5, 0, 1, 2, 3]


def test_synth_network_shape():
    pks, st = eb.synth.network(1000)
    assert len(set(pks)) == 1000 and st.dtype == np.uint64
    assert int(st.max()) >= 15_000_000_000_000_000 and int(st.min()) >= 10**9
    strs = [gs.b58encode(p) for p in pks]
    assert strs == sorted(strs)
