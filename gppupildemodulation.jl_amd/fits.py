"""FITS output of processmetrology: the METROLOGY binary table and its header
written the way the reference's FITSIO/CFITSIO calls lay them out (src/GPPupilDemodulation.jl:
174-189, 239-253 build the keywords and columns; src/FitsUtils.jl:61-156 writes the HDUs), plus
a reader for the same subset (round trips in tests/test_fits.py, and reading METROLOGY tables of
exposures).

The image has no CFITSIO, FITSIO or astropy, so this is a small numpy restatement of the FITS
standard's parts the path uses — an empty primary HDU (FitsUtils.jl:40-58 creates it with
BITPIX 16, NAXIS 0), one BINTABLE extension per table, 2880-byte blocks, big-endian rows:
- columns: Float32 → E, Float64 → D, Int8 → B with TZERO = -128 (CFITSIO's signed-byte
  convention for Julia's Int8 STATE column), UInt8 → B, Int16/32/64 → I/J/K, Bool → L,
  ComplexF32/64 → C/M; an (N, r) array is one r-vector per row (Julia's r × N column, e.g. VOLT
  80E or 144E with keepraw, ABSA/ARGA/B/PHI/X0/Y0 32E in window mode);
- keywords longer than 8 characters or containing spaces use the HIERARCH convention CFITSIO
  writes ("HIERARCH DEMODULATION SIN AMPLITUDE FT T1 D1 = 1.23…"); floats with 15 significant
  digits as CFITSIO's ffd2e does (so values round-trip to ~1e-15 relative, not bit for bit),
  integers and logicals right-justified to column 30, strings quoted.
The column order is the table's insertion order (the reference's Dict order is unspecified).
This is host I/O beside the GPU path, not part of it."""
from __future__ import annotations

import numpy as np

BLOCK = 2880
CARD = 80

_TFORM = {np.dtype(np.float32): "E", np.dtype(np.float64): "D", np.dtype(np.uint8): "B",
          np.dtype(np.int8): "B", np.dtype(np.int16): "I", np.dtype(np.int32): "J",
          np.dtype(np.int64): "K", np.dtype(np.bool_): "L", np.dtype(np.complex64): "C",
          np.dtype(np.complex128): "M", np.dtype(np.uint16): "I", np.dtype(np.uint32): "J",
          np.dtype(np.uint64): "K"}
_CODE = {"E": ">f4", "D": ">f8", "B": "u1", "I": ">i2", "J": ">i4", "K": ">i8", "L": "S1",
         "C": ">c8", "M": ">c16"}
# the standard's unsigned-integer convention (CFITSIO writes it for UInt16/32/64 columns):
# stored signed value + TZERO; flipping the sign bit is exactly that offset
_UNSIGNED = {"I": (np.uint16, np.int16, 1 << 15), "J": (np.uint32, np.int32, 1 << 31),
             "K": (np.uint64, np.int64, 1 << 63)}
# bytes per repeat of the column types read as raw bytes (variable-length descriptors, bits)
_RAW_WIDTH = {"P": 8, "Q": 16}
_STRUCTURAL = ("SIMPLE", "XTENSION", "BITPIX", "NAXIS", "PCOUNT", "GCOUNT", "TFIELDS", "EXTEND",
               "TTYPE", "TFORM", "TZERO", "TSCAL", "TDIM", "TUNIT", "EXTNAME", "END",
               # column-bound or content-bound cards CFITSIO reserves: a re-encoded table gets
               # new column numbers and new data, so old TDISPn / TNULLn / THEAP and the
               # checksums of the old bytes would be wrong (FITSIO's write_header drops them)
               "TDISP", "TNULL", "THEAP", "CHECKSUM", "DATASUM")
COMMENTARY = "__commentary__"  # header key of the COMMENT / HISTORY cards (raw 80-char cards)


def _is_structural(key: str) -> bool:
    return key == COMMENTARY or any(
        key == s or (key.startswith(s) and key[len(s):].isdigit()) for s in _STRUCTURAL)


def _commentary_cards(header: dict | None) -> list[str]:
    return list((header or {}).get(COMMENTARY, []))


def format_float(v: float) -> str:
    """CFITSIO's ffd2e with 15 significant digits (FITSIO's Float64 keywords): %.15G, with a
    decimal point always present."""
    s = "%.15G" % v
    if not np.isfinite(v):
        raise ValueError(f"FITS keywords cannot hold {v!r}")
    if "." not in s:
        s = s.replace("E", ".E") if "E" in s else s + "."
    return s


def _value(v) -> str:
    if isinstance(v, (bool, np.bool_)):
        return "%20s" % ("T" if v else "F")
    if isinstance(v, (int, np.integer)):
        return "%20d" % int(v)
    if isinstance(v, (float, np.floating)):
        return "%20s" % format_float(float(v))
    if isinstance(v, str):
        q = "'" + v.replace("'", "''").ljust(8) + "'"
        return q
    raise TypeError(f"unsupported keyword value {v!r}")


def card(key: str, value=None, comment: str | None = None) -> str:
    """One 80-character header card."""
    if key in ("COMMENT", "HISTORY", ""):
        text = key.ljust(8) + str(value or "")
    elif len(key) <= 8 and " " not in key and key == key.upper():
        text = key.ljust(8) + "= " + _value(value)
    else:
        v = _value(value).strip() if not isinstance(value, str) else _value(value)
        text = f"HIERARCH {key} = {v}"
    if comment:
        text += " / " + comment
    if len(text) > CARD:
        if comment:
            return card(key, value)
        raise ValueError(f"keyword card longer than 80 characters: {text!r}")
    if not text.isascii():
        raise ValueError(f"non-ASCII header card: {text!r}")
    return text.ljust(CARD)


def _header_bytes(cards: list[str]) -> bytes:
    raw = "".join(cards) + "END".ljust(CARD)
    raw += " " * (-len(raw) % BLOCK)
    return raw.encode("ascii")


def _columns(table: dict):
    """(name, tform, tzero, big-endian field dtype, data as field values) per column."""
    n = None
    cols = []
    for name, a in table.items():
        a = np.asarray(a)
        if a.ndim == 0 or a.ndim > 2:
            raise ValueError(f"column {name}: (N,) or (N, r) arrays only, got shape {a.shape}")
        if n is None:
            n = a.shape[0]
        elif a.shape[0] != n:
            raise ValueError(f"column {name}: {a.shape[0]} rows, expected {n}")
        if a.dtype.kind == "S" and a.ndim == 1:  # character column rA
            r = max(a.dtype.itemsize, 1)
            cols.append((name, f"{r}A", None, np.dtype(f"S{r}"), a))
            continue
        if a.dtype not in _TFORM:
            raise TypeError(f"column {name}: unsupported dtype {a.dtype}")
        letter = _TFORM[a.dtype]
        r = 1 if a.ndim == 1 else a.shape[1]
        tzero = None
        if a.dtype == np.int8:
            tzero = -128
            a = (a.astype(np.int16) + 128).astype(np.uint8)
        elif a.dtype.kind == "u" and letter in _UNSIGNED:
            ut, st, off = _UNSIGNED[letter]
            tzero = off
            a = (a ^ ut(off)).view(st)
        elif a.dtype == np.bool_:
            a = np.where(a, b"T", b"F")
        fdt = np.dtype(_CODE[letter]) if a.ndim == 1 else np.dtype((_CODE[letter], (r,)))
        cols.append((name, f"{r}{letter}", tzero, fdt, a))
    return n or 0, cols


def bintable_hdu(table: dict, header: dict | None = None, *, extname: str | None = None,
                 units: dict | None = None) -> bytes:
    """One BINTABLE extension (header + data blocks)."""
    n, cols = _columns(table)
    rec = np.dtype([(name, fdt) for name, _, _, fdt, _ in cols])
    data = np.zeros(n, dtype=rec)
    for name, _, _, _, a in cols:
        data[name] = a
    cards = [card("XTENSION", "BINTABLE"), card("BITPIX", 8), card("NAXIS", 2),
             card("NAXIS1", rec.itemsize), card("NAXIS2", n), card("PCOUNT", 0),
             card("GCOUNT", 1), card("TFIELDS", len(cols))]
    for i, (name, tform, tzero, _, _) in enumerate(cols, 1):
        cards += [card(f"TTYPE{i}", name), card(f"TFORM{i}", tform)]
        if tzero is not None:
            cards.append(card(f"TZERO{i}", tzero))
        if units and name in units:
            cards.append(card(f"TUNIT{i}", units[name]))
    if extname is not None:
        cards.append(card("EXTNAME", extname))
    for k, v in (header or {}).items():
        if not _is_structural(k):
            cards.append(card(k, v))
    cards += _commentary_cards(header)
    body = data.tobytes()
    body += b"\0" * (-len(body) % BLOCK)
    return _header_bytes(cards) + body


def primary_hdu(header: dict | None = None) -> bytes:
    """The empty primary HDU (FitsUtils.jl:40-58: BITPIX 16, NAXIS 0) with the given keywords."""
    cards = [card("SIMPLE", True), card("BITPIX", 16), card("NAXIS", 0), card("EXTEND", True)]
    for k, v in (header or {}).items():
        if not _is_structural(k):
            cards.append(card(k, v))
    return _header_bytes(cards + _commentary_cards(header))


_BITPIX_DTYPE = {8: "u1", 16: ">i2", 32: ">i4", 64: ">i8", -32: ">f4", -64: ">f8"}
_DTYPE_BITPIX = {np.dtype(np.uint8): 8, np.dtype(np.int16): 16, np.dtype(np.int32): 32,
                 np.dtype(np.int64): 64, np.dtype(np.float32): -32, np.dtype(np.float64): -64}


def image_hdu(data, header: dict | None = None, *, primary: bool = False,
              extname: str | None = None) -> bytes:
    """An image HDU (primary or IMAGE extension); data None gives the empty HDU.  numpy's C-order
    shape (…, n2, n1) is NAXIS1 = n1 (Julia's column-major (n1, n2, …) array)."""
    if data is None:
        bitpix, shape, body = 16, (), b""
    else:
        data = np.asarray(data)
        if data.dtype not in _DTYPE_BITPIX:
            raise TypeError(f"unsupported image dtype {data.dtype}")
        bitpix, shape = _DTYPE_BITPIX[data.dtype], data.shape
        body = np.ascontiguousarray(data, dtype=_BITPIX_DTYPE[bitpix]).tobytes()
        body += b"\0" * (-len(body) % BLOCK)
    cards = [card("SIMPLE", True) if primary else card("XTENSION", "IMAGE"),
             card("BITPIX", bitpix), card("NAXIS", len(shape))]
    cards += [card(f"NAXIS{j}", n) for j, n in enumerate(reversed(shape), 1)]
    cards += [card("EXTEND", True)] if primary else [card("PCOUNT", 0), card("GCOUNT", 1)]
    if extname is not None and not primary:
        cards.append(card("EXTNAME", extname))
    for k, v in (header or {}).items():
        if not _is_structural(k):
            cards.append(card(k, v))
    return _header_bytes(cards + _commentary_cards(header)) + body


def write_fits(path: str, hdus) -> None:
    """hdus: [(header, data)] — data None or an ndarray (image; the first HDU is the primary),
    or a dict of columns (BINTABLE; a table first gets an empty primary HDU before it).  The
    EXTNAME of each header is kept."""
    with open(path, "wb") as f:
        for j, (hdr, data) in enumerate(hdus):
            hdr = dict(hdr or {})
            name = hdr.get("EXTNAME")
            if isinstance(data, dict):
                if j == 0:
                    f.write(primary_hdu())
                f.write(bintable_hdu(data, hdr, extname=name, units=_units_of(hdr)))
            else:
                f.write(image_hdu(data, hdr, primary=j == 0, extname=name))


def _units_of(hdr: dict) -> dict:
    """{column name: unit} from TTYPEn / TUNITn (FitsUtils.getunits, src/FitsUtils.jl:14-25)."""
    return {hdr[f"TTYPE{k[5:]}"]: v for k, v in hdr.items()
            if k.startswith("TUNIT") and k[5:].isdigit() and f"TTYPE{k[5:]}" in hdr}


def fits_copy(dst: str, src: str, content: dict | None = None,
              headers: dict | None = None) -> None:
    """FitsUtils.FITScopy!(dst, src, content, header) (src/FitsUtils.jl:96-154): every HDU of src
    copied to dst, the HDUs named in `content` / `headers` (EXTNAME → table dict or array /
    header dict) replaced, names absent from src appended after it.  HDUs that are not replaced
    are copied byte for byte (any column type, scaling, checksum or commentary card stays as the
    source holds it).  A replaced table keeps the source's TUNITs and COMMENT/HISTORY cards; a
    header-only replacement keeps the source's column cards and data bytes."""
    content, headers = dict(content or {}), dict(headers or {})
    raw = _read_raw(src)
    out = []
    for a, hb, e, hdr in _hdu_spans(raw):
        name = hdr.get("EXTNAME")
        if name is None or (name not in content and name not in headers):
            out.append(raw[a:e])
            continue
        h = headers.pop(name, hdr)
        if COMMENTARY not in h and hdr.get(COMMENTARY):
            h = dict(h, **{COMMENTARY: hdr[COMMENTARY]})
        if name in content:
            d = content.pop(name)
            if isinstance(d, dict) and "TFIELDS" in hdr and h is not hdr:
                h = {**{k: v for k, v in hdr.items()
                        if k.startswith("TUNIT") or k.startswith("TTYPE")}, **h}
            h = dict(h, EXTNAME=name)
            if isinstance(d, dict):
                out.append(bintable_hdu(d, h, extname=name, units=_units_of(h)))
            else:
                out.append(image_hdu(d, h, primary=a == 0, extname=name))
            continue
        # header only: the source's structural / column cards and its data bytes, new keywords
        keep = [raw[j:j + CARD].decode("ascii") for j in range(a, hb, CARD)]
        keep = [c for c in keep if _card_key(c) is not None and _is_structural(_card_key(c))
                and _card_key(c) not in ("END", "CHECKSUM", "DATASUM")]
        cards = keep + [card(k, v) for k, v in h.items() if not _is_structural(k)]
        out.append(_header_bytes(cards + _commentary_cards(h)) + raw[hb:e])
    for name, d in content.items():
        h = dict(headers.pop(name, {}), EXTNAME=name)
        out.append(bintable_hdu(d, h, extname=name, units=_units_of(h)) if isinstance(d, dict)
                   else image_hdu(d, h, extname=name))
    for name, h in headers.items():
        out.append(image_hdu(None, dict(h, EXTNAME=name), extname=name))
    with open(dst, "wb") as f:
        for b in out:
            f.write(b)


def write_metrology(path: str, table: dict, header: dict, *, primary_header: dict | None = None,
                    units: dict | None = None, extname: str = "METROLOGY") -> None:
    """processmetrology's (table, hdr) as a FITS file: primary HDU + the METROLOGY table."""
    with open(path, "wb") as f:
        f.write(primary_hdu(primary_header))
        f.write(bintable_hdu(table, header, extname=extname, units=units))


# ------------------------------------------------------------------------------- reading
def _parse_value(s: str):
    s = s.strip()
    if s.startswith("'"):
        out, i = [], 1
        while i < len(s):
            if s[i] == "'":
                if i + 1 < len(s) and s[i + 1] == "'":
                    out.append("'")
                    i += 2
                    continue
                break
            out.append(s[i])
            i += 1
        return "".join(out).rstrip()
    s = s.split("/", 1)[0].strip()
    if s in ("T", "F"):
        return s == "T"
    if s == "":
        return None
    try:
        return int(s)
    except ValueError:
        return float(s.replace("D", "E"))


def parse_card(text: str):
    """(key, value) of one card; (None, None) for commentary and blank cards."""
    if text.startswith("HIERARCH "):
        key, _, rest = text[9:].partition("=")
        return key.strip(), _parse_value(rest)
    key = text[:8].strip()
    if text[8:10] != "= " or key in ("COMMENT", "HISTORY", ""):
        return None, None
    return key, _parse_value(text[10:])


def _card_key(text: str):
    if text.startswith("HIERARCH "):
        return text[9:].partition("=")[0].strip()
    key = text[:8].strip()
    if key == "END":
        return key
    return key if text[8:10] == "= " else None


def _read_raw(path: str) -> bytes:
    if str(path).endswith(".gz"):  # the reference's SUFFIXES include .fits.gz (CFITSIO reads it)
        import gzip
        with gzip.open(path, "rb") as f:
            return f.read()
    with open(path, "rb") as f:
        return f.read()


def _data_size(hdr: dict) -> int:
    if hdr.get("XTENSION") == "BINTABLE":
        return hdr["NAXIS2"] * hdr["NAXIS1"] + hdr.get("PCOUNT", 0)
    n = hdr.get("NAXIS", 0)
    if n == 0:
        return 0
    count = int(np.prod([hdr[f"NAXIS{j}"] for j in range(1, n + 1)]))
    return (count * abs(hdr["BITPIX"]) // 8 + hdr.get("PCOUNT", 0)) * hdr.get("GCOUNT", 1)


def _hdu_spans(raw: bytes):
    """(start, end of header, end of data, header dict) of every HDU; the header dict holds the
    COMMENT / HISTORY cards as raw text under COMMENTARY."""
    pos = 0
    while pos < len(raw):
        a, hdr, comm, done = pos, {}, [], False
        while not done:
            block = raw[pos:pos + BLOCK].decode("ascii")
            pos += BLOCK
            for j in range(0, BLOCK, CARD):
                c = block[j:j + CARD]
                if c.startswith("END") and c[3:].strip() == "":
                    done = True
                    break
                k, v = parse_card(c)
                if k is not None:
                    hdr[k] = v
                elif c[:8].strip() in ("COMMENT", "HISTORY"):
                    comm.append(c)
        if comm:
            hdr[COMMENTARY] = comm
        size = _data_size(hdr)
        e = pos + size + (-size % BLOCK)
        yield a, pos, e, hdr
        pos = e


def _column(a, hdr: dict, i: int, letter: str):
    """Field values of column i with the header's TZERO / TSCAL applied as CFITSIO does
    (Int8 and unsigned-integer offsets exactly, other scalings as Float64)."""
    tz, ts = hdr.get(f"TZERO{i}"), hdr.get(f"TSCAL{i}", 1)
    a = a.astype(a.dtype.newbyteorder("="))
    if tz is None and ts == 1:
        return a
    if letter == "B" and tz == -128 and ts == 1:
        return (a.astype(np.int16) - 128).astype(np.int8)
    if letter in _UNSIGNED and ts == 1 and tz == _UNSIGNED[letter][2]:
        ut, _, off = _UNSIGNED[letter]
        return a.view(ut) ^ ut(off)
    return a.astype(np.float64) * ts + (tz or 0)


def read_fits(path: str):
    """[(header dict, data)] per HDU (path may be gzip-compressed, .gz): None for an empty HDU,
    an ndarray for an image, a dict of columns for a BINTABLE ((N,) or (N, r) arrays in native
    byte order, TZERO/TSCAL applied: Int8 and UInt16/32/64 offsets exactly; variable-length
    (P/Q) descriptors and bit (X) columns as raw bytes, the heap not read)."""
    raw = _read_raw(path)
    hdus = []
    for _, pos, _, hdr in _hdu_spans(raw):
        data = None
        if hdr.get("XTENSION") == "BINTABLE":
            n, width, k = hdr["NAXIS2"], hdr["NAXIS1"], hdr["TFIELDS"]
            fields, letters = [], []
            for i in range(1, k + 1):
                tform = hdr[f"TFORM{i}"].strip()
                letter = tform.lstrip("0123456789")[:1]
                rs = tform[:len(tform) - len(tform.lstrip("0123456789"))]
                r = int(rs) if rs else 1
                letters.append(letter)
                name = hdr.get(f"TTYPE{i}", f"COL{i}")
                if letter == "A":
                    fields.append((name, f"S{r}"))
                elif letter in _CODE:
                    fields.append((name, _CODE[letter] if r == 1 else (_CODE[letter], (r,))))
                elif letter in _RAW_WIDTH or letter == "X":
                    nb = r * _RAW_WIDTH[letter] if letter in _RAW_WIDTH else (r + 7) // 8
                    fields.append((name, f"V{nb}"))
                else:
                    raise NotImplementedError(f"TFORM {tform} (column {name})")
            rec = np.dtype(fields)
            if rec.itemsize != width:
                raise ValueError(f"NAXIS1 {width} != row size {rec.itemsize}")
            rows = np.frombuffer(raw, dtype=rec, count=n, offset=pos)
            data = {}
            for i, ((name, _), letter) in enumerate(zip(fields, letters), 1):
                a = rows[name]
                if letter == "L":
                    a = a == b"T"
                elif a.dtype.kind in "SV":
                    a = a.copy()
                else:
                    a = _column(a, hdr, i, letter)
                data[name] = a
        elif hdr.get("NAXIS", 0) != 0:  # image: raw values, BZERO/BSCALE left in the header
            shape = tuple(hdr[f"NAXIS{j}"] for j in range(hdr["NAXIS"], 0, -1))
            dt = np.dtype(_BITPIX_DTYPE[hdr["BITPIX"]])
            img = np.frombuffer(raw, dtype=dt, count=int(np.prod(shape)), offset=pos)
            data = img.reshape(shape).astype(dt.newbyteorder("="))
        hdus.append((hdr, data))
    return hdus
