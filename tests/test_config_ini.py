"""INI reader (include/nxec.h §8) against the reference's own sample
storage_class.ini (tests/golden/sample/, copied verbatim: config 1's literal
RS(4,2) reading) and its proxy.ini [misc] keys; then Config's
edge cases (config.cc:267-282 one default class, :664-705 defaults and
bounds, :320 the CAR flag).  CPU only: no compute call."""
import os

import pytest

from nexoedge_amd import _lib, nxec

SAMPLE = os.path.join(os.path.dirname(__file__), "golden", "sample")


def test_reference_sample_storage_class():
    classes = nxec.storage_classes(os.path.join(SAMPLE, "storage_class.ini"))
    assert classes == [{"name": "standard", "coding": "rs", "n": 4, "k": 2, "f": 1, "max_chunk_size": 4 << 20,
                        "default": True}]
    # config 1's literal reading: a 4 MiB file in one stripe of k = 2 chunks of
    # ceil(4 MiB / 2) = 2 MiB (rs.cc:52-55 getChunkSize), n = 4 chunks
    c = classes[0]
    ns, nf, cs_last = nxec.object_layout(c["n"], c["k"], 4 << 20, c["max_chunk_size"])
    assert (ns, cs_last) == (1, 2 << 20)


def test_reference_sample_proxy_car_flag():
    assert nxec.proxy_repair_using_car(os.path.join(SAMPLE, "proxy.ini")) is False


def write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_config_edge_cases(tmp_path):
    p = write(tmp_path, "sc.ini", "[a]\ndefault = 0\ncoding = RS\nn = 0\nk = -4\nmax_chunk_size = 2000000000\n"
                                  "f = 99999999999\n[b]\ndefault = true\ncoding = lrc\n")
    a, b = nxec.storage_classes(p)
    assert (a["coding"], a["n"], a["k"], a["f"], a["max_chunk_size"]) == ("rs", 0, 0, -1, 1 << 30)
    assert (b["coding"], b["n"], b["k"], b["f"], b["max_chunk_size"], b["default"]) == ("unknown", -1, -1, -1, 0, True)
    for bad in ("[a]\ndefault = 1\n[b]\ndefault = 1\n",    # two default classes
                "[a]\nn = 4\n",                              # no default key
                "[a]\ndefault = 1\nnot a pair\n",            # malformed line
                "[a]\ndefault = 1\n[a]\ndefault = 0\n",      # duplicate section
                "n = 4\n[a]\ndefault = 1\n"):                # key outside a section
        with pytest.raises(_lib.NxecError):
            nxec.storage_classes(write(tmp_path, "bad.ini", bad))
    assert nxec.proxy_repair_using_car(write(tmp_path, "p.ini", "[misc]\nrepair_using_car = true\n")) is True
    with pytest.raises(_lib.NxecError):
        nxec.proxy_repair_using_car(write(tmp_path, "p2.ini", "[misc]\nrepair_using_car = maybe\n"))
    with pytest.raises(_lib.NxecError):
        nxec.storage_classes(str(tmp_path / "missing.ini"))
