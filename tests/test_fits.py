"""FITS output of processmetrology (§8f rank 4; src/GPPupilDemodulation.jl:174-189, 239-253,
src/FitsUtils.jl:40-156): the METROLOGY table and its keywords written in the layout FITSIO /
CFITSIO give them, read back by the same module.  No FITS library exists in the image, so the
layout is checked against the FITS standard directly (2880-byte blocks, 80-character cards,
HIERARCH keywords, TFORM / TZERO, big-endian rows); parity with a CFITSIO-written file is
unpinned (no such file in the reference)."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def fits():
    import gpdemod_loader
    return gpdemod_loader.load().fits


def _window_table(N=1000, seed=5, fitoffsets=True, keepraw=False):
    """A window-mode processmetrology table: TIME, VOLT (80 or 144 per row), the per-sample
    Float32 parameter columns (N, 32), STATE (Int8, TRANSIENT = -1 included)."""
    rng = np.random.default_rng(seed)
    tab = {"TIME": np.arange(N, dtype=np.int32) * 2000,
           "VOLT": rng.standard_normal((N, 144 if keepraw else 80)).astype(np.float32)}
    for k in (["X0", "Y0"] if fitoffsets else []) + ["ABSA", "ARGA", "B", "PHI"]:
        tab[k] = rng.standard_normal((N, 32)).astype(np.float32)
    tab["STATE"] = rng.integers(-1, 4, N).astype(np.int8)
    tab["STATE"][:3] = [-128, 127, -1]
    return tab


def _header(seed=6):
    rng = np.random.default_rng(seed)
    hdr = {"EXTNAME": "METROLOGY", "MJD-OBS": 58849.123456789, "ESO INS MET MODE": "FAINT",
           "PROCSOFT": "GPPupilDemodulation.jl", "NSAMPLES": 1000, "FLAG": True}
    for side in ("FT", "SC"):
        for tel in range(1, 5):
            for d in ("D1", "D2", "D3", "D4"):
                name = f"{side} T{tel} {d}"
                hdr[f"DEMODULATION AMPLITUDE ABS {name}"] = float(rng.random())
                hdr[f"DEMODULATION AMPLITUDE ARG {name}"] = float(rng.uniform(-np.pi, np.pi))
                hdr[f"DEMODULATION SIN AMPLITUDE {name}"] = float(rng.uniform(0.3, 2.5))
                hdr[f"DEMODULATION SIN PHASE {name}"] = float(rng.uniform(-np.pi, np.pi) * 1e-7)
                hdr[f"DEMODULATION CENTER X0 {name}"] = float(rng.standard_normal() * 1e3)
    return hdr


@pytest.mark.parametrize("keepraw", [False, True])
def test_metrology_table_round_trip(fits, tmp_path, keepraw):
    tab, hdr = _window_table(keepraw=keepraw), _header()
    path = str(tmp_path / "m.fits")
    fits.write_metrology(path, tab, hdr, primary_header={"ESO INS PMC1 MODULATE": True},
                         units={"TIME": "us", "VOLT": "V"})
    raw = open(path, "rb").read()
    assert len(raw) % 2880 == 0
    (h0, d0), (h1, d1) = fits.read_fits(path)
    assert d0 is None and h0["SIMPLE"] is True and h0["BITPIX"] == 16 and h0["NAXIS"] == 0
    assert h0["ESO INS PMC1 MODULATE"] is True
    assert h1["XTENSION"] == "BINTABLE" and h1["EXTNAME"] == "METROLOGY"
    assert h1["NAXIS2"] == 1000 and h1["TFIELDS"] == len(tab)
    assert list(d1) == list(tab)  # insertion order
    for k, a in tab.items():
        assert d1[k].dtype == a.dtype and d1[k].shape == a.shape, k
        assert d1[k].tobytes() == a.tobytes(), k  # Float32 and Int8 bit for bit
    forms = {h1[f"TTYPE{i}"]: h1[f"TFORM{i}"] for i in range(1, h1["TFIELDS"] + 1)}
    assert forms["VOLT"] == ("144E" if keepraw else "80E") and forms["ABSA"] == "32E"
    assert forms["STATE"] == "1B" and forms["TIME"] == "1J"
    i_state = [h1[f"TTYPE{i}"] for i in range(1, h1["TFIELDS"] + 1)].index("STATE") + 1
    assert h1[f"TZERO{i_state}"] == -128
    assert h1["TUNIT1"] == "us" and h1["TUNIT2"] == "V"
    for k, v in hdr.items():
        if isinstance(v, float):
            assert h1[k] == pytest.approx(v, rel=1e-14, abs=0), k  # 15 significant digits
        else:
            assert h1[k] == v, k


def test_header_cards_follow_the_standard(fits, tmp_path):
    hdr = _header()
    path = str(tmp_path / "h.fits")
    fits.write_metrology(path, {"TIME": np.arange(4, dtype=np.float64)}, hdr)
    text = open(path, "rb").read()[2880:]
    cards = []
    for i in range(0, len(text), 80):
        c = text[i:i + 80].decode("ascii")
        if c.rstrip() == "END":
            break
        cards.append(c)
    assert cards[0].startswith("XTENSION= 'BINTABLE'")
    assert all(len(c) == 80 for c in cards)
    hier = [c for c in cards if c.startswith("HIERARCH DEMODULATION SIN AMPLITUDE FT T1 D1 = ")]
    assert len(hier) == 1
    # fixed-format values end in column 30
    naxis2 = next(c for c in cards if c.startswith("NAXIS2  = "))
    assert naxis2[29] == "4" and naxis2[30:].strip() == ""
    assert next(c for c in cards if c.startswith("PROCSOFT= ")).startswith(
        "PROCSOFT= 'GPPupilDemodulation.jl'")


def test_float_keyword_format(fits):
    """CFITSIO's 15 significant digits with a decimal point."""
    assert fits.format_float(1.0) == "1."
    assert fits.format_float(0.1) == "0.1"
    assert fits.format_float(1e20) == "1.E+20"
    assert fits.format_float(-1.23456789012345678e-7) == "-1.23456789012346E-07"
    with pytest.raises(ValueError):
        fits.format_float(float("nan"))
    with pytest.raises(ValueError):
        fits.card("DEMODULATION AMPLITUDE ABS FT T1 D1 WITH A VERY LONG NAME THAT OVERFLOWS", 1.5)


def test_processmetrology_header_written(fits, tmp_path):
    """processmetrology's own keyword names (built by demod.py) survive the file: 6 per diode
    with fitoffsets, 4 without, and PROCSOFT."""
    import gpdemod_loader
    gpd = gpdemod_loader.load()
    keys = []
    for side, tel, diode in gpd.demod._diode_order():
        name = f"{side.name} T{tel} {diode.name}"
        keys += [f"DEMODULATION CENTER X0 {name}", f"DEMODULATION SIN PHASE {name}"]
    hdr = {k: 0.5 for k in keys}
    hdr["PROCSOFT"] = "GPPupilDemodulation.jl"
    path = str(tmp_path / "p.fits")
    fits.write_metrology(path, {"VOLT": np.zeros((2, 80), np.float32)}, hdr)
    (_, _), (h1, d1) = fits.read_fits(path)
    assert all(h1[k] == 0.5 for k in keys) and h1["PROCSOFT"] == "GPPupilDemodulation.jl"
    assert d1["VOLT"].shape == (2, 80)


def test_exposure_copy_replaces_the_metrology_table(fits, tmp_path):
    """FITScopy!(dst, src, "METROLOGY" => table, "METROLOGY" => hdr) (src/FitsUtils.jl:96-154,
    called by the reference's main loop): every other HDU — images, other tables with
    character columns, header keywords — copied unchanged; METROLOGY replaced, its TUNITs kept."""
    rng = np.random.default_rng(9)
    img = rng.integers(-300, 300, (6, 5)).astype(np.int16)
    cube = rng.standard_normal((2, 3, 4)).astype(np.float32)
    tel = {"TEL_NAME": np.array([b"UT1", b"UT2", b"UT3", b"UT4"]),
           "STA_INDEX": np.arange(4, dtype=np.int16)}
    met = {"TIME": np.arange(10, dtype=np.int32), "VOLT": rng.standard_normal((10, 80)).astype(np.float32)}
    src, dst = str(tmp_path / "src.fits"), str(tmp_path / "dst.fits")
    fits.write_fits(src, [({"ESO INS PMC1 MODULATE": True, "MJD-OBS": 58849.5}, img),
                          ({"EXTNAME": "OI_ARRAY", "ARRNAME": "VLTI"}, tel),
                          ({"EXTNAME": "IMAGING_DATA", "BZERO": 0.0}, cube),
                          ({"EXTNAME": "METROLOGY", "TUNIT1": "us", "TTYPE1": "TIME",
                            "TTYPE2": "VOLT"}, met)])
    hdus = fits.read_fits(src)
    assert [h.get("EXTNAME") for h, _ in hdus] == [None, "OI_ARRAY", "IMAGING_DATA", "METROLOGY"]
    np.testing.assert_array_equal(hdus[0][1], img)
    np.testing.assert_array_equal(hdus[2][1], cube)
    assert list(hdus[1][1]["TEL_NAME"]) == [b"UT1", b"UT2", b"UT3", b"UT4"]
    assert hdus[3][0]["TUNIT1"] == "us"
    new = dict(met, VOLT=(met["VOLT"] * 2).astype(np.float32), B=np.ones((10, 32), np.float32))
    newhdr = dict(hdus[3][0], PROCSOFT="GPPupilDemodulation.jl")
    fits.fits_copy(dst, src, {"METROLOGY": new}, {"METROLOGY": newhdr, "EXTRA": {"X": 1}})
    out = fits.read_fits(dst)
    assert [h.get("EXTNAME") for h, _ in out] == [None, "OI_ARRAY", "IMAGING_DATA", "METROLOGY",
                                                  "EXTRA"]
    assert out[0][0] == hdus[0][0] and out[1][0] == hdus[1][0] and out[2][0] == hdus[2][0]
    np.testing.assert_array_equal(out[0][1], img)
    np.testing.assert_array_equal(out[2][1], cube)
    for k in tel:
        np.testing.assert_array_equal(out[1][1][k], tel[k])
    h3, d3 = out[3]
    assert h3["PROCSOFT"] == "GPPupilDemodulation.jl" and h3["TUNIT1"] == "us"
    assert d3["VOLT"].tobytes() == new["VOLT"].tobytes() and d3["B"].shape == (10, 32)
    assert out[4][0]["X"] == 1 and out[4][1] is None


def test_gzip_input(fits, tmp_path):
    """.fits.gz exposures (the reference's SUFFIXES, src/GPPupilDemodulation.jl:14) read as is."""
    import gzip
    tab = _window_table(N=50)
    p = str(tmp_path / "a.fits")
    fits.write_metrology(p, tab, {"X": 1})
    with open(p, "rb") as f, gzip.open(p + ".gz", "wb") as g:
        g.write(f.read())
    (_, _), (h, d) = fits.read_fits(p + ".gz")
    assert h["X"] == 1 and all(d[k].tobytes() == tab[k].tobytes() for k in tab)


def _hdu(fits, cards, body=b""):
    body = body + b"\0" * (-len(body) % fits.BLOCK)
    return fits._header_bytes([c if len(c) == 80 else fits.card(*c) for c in cards]) + body


def test_copy_keeps_untouched_hdus_byte_for_byte(fits, tmp_path):
    """FITScopy! passes every HDU it does not replace through CFITSIO unchanged: an unsigned
    (TZERO = 32768) column, a variable-length (P) column with its heap and a CHECKSUM card in an
    unrelated table come out byte for byte.  The replaced METROLOGY table drops the old
    CHECKSUM/DATASUM and column-bound TDISPn/TNULLn (new columns, new bytes) and keeps its
    COMMENT/HISTORY cards; a header-only replacement keeps the data bytes."""
    import struct
    rows = b"".join(struct.pack(">iiH", 2, 2 * j, u ^ 0x8000) for j, u in enumerate((0, 40000, 65535)))
    heap = bytes([1, 2, 3, 4, 5, 6])
    other = _hdu(fits, [("XTENSION", "BINTABLE"), ("BITPIX", 8), ("NAXIS", 2), ("NAXIS1", 10),
                        ("NAXIS2", 3), ("PCOUNT", len(heap)), ("GCOUNT", 1), ("TFIELDS", 2),
                        ("TTYPE1", "VARCOL"), ("TFORM1", "1PB(2)"), ("TTYPE2", "U"),
                        ("TFORM2", "1I"), ("TZERO2", 32768), ("EXTNAME", "OI_OTHER"),
                        ("CHECKSUM", "9aJ5AaG49aG4AaG4"), ("DATASUM", "12345")], rows + heap)
    met = {"TIME": np.arange(4, dtype=np.int32), "VOLT": np.ones((4, 80), np.float32)}
    mb = fits.bintable_hdu(met, {"TUNIT1": "us"}, extname="METROLOGY", units={"TIME": "us"})
    hdr_end = mb.index(b"END" + b" " * 77)
    extra = "".join(fits.card(*c) for c in [("TDISP2", "E15.7"), ("TNULL1", -1),
                                            ("CHECKSUM", "0000000000000000"), ("DATASUM", "42")])
    extra += fits.card("COMMENT", "metrology of the four telescopes")
    extra += fits.card("HISTORY", "written by the instrument")
    mb = mb[:hdr_end] + extra.encode() + mb[hdr_end:]
    # re-block the header (the inserted cards may overflow its last block)
    cards = [mb[j:j + 80].decode() for j in range(0, mb.index(b"END" + b" " * 77), 80)]
    data_at = (mb.index(b"END" + b" " * 77) // 2880 + 1) * 2880
    mb = _hdu(fits, cards, mb[data_at:].rstrip(b"\0") or b"")
    src, dst, dst2 = (str(tmp_path / n) for n in ("s.fits", "d.fits", "h.fits"))
    with open(src, "wb") as f:
        f.write(fits.primary_hdu({"MJD-OBS": 58849.5}) + other + mb)
    hdus = fits.read_fits(src)
    u = hdus[1][1]["U"]
    assert u.dtype == np.uint16 and list(u) == [0, 40000, 65535]
    assert hdus[1][1]["VARCOL"].dtype.kind == "V"
    h_met = hdus[2][0]
    assert h_met["CHECKSUM"] == "0000000000000000" and len(h_met[fits.COMMENTARY]) == 2
    new = dict(met, B=np.zeros((4, 32), np.float32))
    fits.fits_copy(dst, src, {"METROLOGY": new}, {"METROLOGY": dict(h_met, PROCSOFT="x")})
    raw_src, raw_dst = open(src, "rb").read(), open(dst, "rb").read()
    assert raw_dst[:2880 + len(other)] == raw_src[:2880 + len(other)]  # primary + OI_OTHER
    out = fits.read_fits(dst)
    h3, d3 = out[2]
    for k in ("CHECKSUM", "DATASUM", "TDISP2", "TNULL1"):
        assert k not in h3, k
    assert h3["PROCSOFT"] == "x" and h3["TUNIT1"] == "us"
    assert [c[:8].strip() for c in h3[fits.COMMENTARY]] == ["COMMENT", "HISTORY"]
    assert d3["B"].shape == (4, 32) and list(out[1][1]["U"]) == [0, 40000, 65535]
    # header-only replacement: the column cards and the data bytes of the source
    fits.fits_copy(dst2, src, None, {"OI_OTHER": {"ARRNAME": "VLTI"}})
    o2 = fits.read_fits(dst2)
    assert o2[1][0]["ARRNAME"] == "VLTI" and o2[1][0]["TZERO2"] == 32768
    assert "CHECKSUM" not in o2[1][0]
    assert list(o2[1][1]["U"]) == [0, 40000, 65535]
    assert o2[1][1]["VARCOL"].tobytes() == hdus[1][1]["VARCOL"].tobytes()
    raw2 = open(dst2, "rb").read()
    assert raw2[-len(mb):] == raw_src[-len(mb):]  # METROLOGY untouched this time: byte for byte


def test_unsigned_columns_round_trip(fits, tmp_path):
    """UInt16/32/64 columns are written with the standard TZERO offsets and read back exactly."""
    tab = {"A": np.array([0, 1, 65535], np.uint16), "B": np.array([0, 2**31, 2**32 - 1], np.uint32),
           "C": np.array([0, 2**63, 2**64 - 1], np.uint64)}
    p = str(tmp_path / "u.fits")
    fits.write_metrology(p, tab, {})
    (_, _), (h, d) = fits.read_fits(p)
    assert (h["TZERO1"], h["TZERO2"], h["TZERO3"]) == (32768, 2**31, 2**63)
    for k in tab:
        assert d[k].dtype == tab[k].dtype and np.array_equal(d[k], tab[k]), k
