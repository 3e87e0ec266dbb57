"""Native JSON encoder (native/jsonenc.cpp) is byte-identical to
jdumps(separators=(",", ":"), ensure_ascii=False) -- the compact, UTF-8 text the
reference's Jackson writes for map values on topics."""
import collections
import functools
import json
import random
import struct

import numpy as np
import pytest

from langstream_amd.utils import fastjson

jdumps = functools.partial(json.dumps, separators=(",", ":"), ensure_ascii=False)


def test_floats_match_repr():
    rnd = random.Random(7)
    vals = [0.0, -0.0, 1.0, -1.0, 1e16, 1e15, 1.5e16, 1e-5, 1e-4, 1.234e-4, 123.0, 1e22, 5e-324,
            1.7976931348623157e308, float("nan"), float("inf"), -float("inf"), 0.1, 9999999999999998.0]
    for _ in range(20000):
        vals.append(rnd.uniform(-1, 1) * 10 ** rnd.randint(-30, 30))
        vals.append(float(np.float32(rnd.gauss(0, 1))))
        vals.append(struct.unpack("d", struct.pack("Q", rnd.getrandbits(64)))[0])
    assert [fastjson.dumps(v) for v in vals] == [jdumps(v) for v in vals]


def test_structures_and_strings():
    objs = [{"a": [1, 2, {"b": None, "c": True}], "é": "ünï \U0001f600\x7f\x00\"\\\n\t\r\b\f", 3: 4, 2.5: 1,
             None: 0, False: 1},
            [], {}, (1, 2), [10 ** 30, -10 ** 30, -5, 0], "x" * 1000, {"k": [[[]]]}, "汉字",
            {"embeddings": np.random.default_rng(0).standard_normal(384).astype(np.float32).tolist()}]
    for o in objs:
        assert fastjson.dumps(o) == jdumps(o)
    assert fastjson.dumps(collections.OrderedDict(a=1, b=[1.5])) == jdumps(collections.OrderedDict(a=1, b=[1.5]))


def test_unsupported_falls_back_to_json_errors():
    class Foo:
        pass
    with pytest.raises(TypeError):
        fastjson.dumps({"a": Foo()})
    cyc = []
    cyc.append(cyc)
    with pytest.raises(ValueError):
        fastjson.dumps(cyc)


def test_kafka_native_records_match_python():
    from langstream_amd.topics.kafka import protocol as P
    if P._ENC is None:
        pytest.skip("native runtime not built")
    rnd = random.Random(3)
    recs = []
    for i in range(300):
        k = None if i % 7 == 0 else bytes(rnd.getrandbits(8) for _ in range(rnd.randint(0, 40)))
        v = None if i % 11 == 0 else bytes(rnd.getrandbits(8) for _ in range(rnd.randint(0, 3000)))
        hs = [("h%d" % j, None if j == 1 else b"x" * j) for j in range(i % 4)]
        hs += [("ünï", b"\x00\xff")] if i % 5 == 0 else []
        recs.append((k, v, hs, 1700000000000 + rnd.randint(-5000, 5000)))
    assert P._ENC(recs, recs[0][3]) == bytes(P._encode_records_py(recs, recs[0][3]))
    batch = P.encode_batch(100, recs)
    native = list(P.decode_batches(batch, verify_crc=True))
    assert native == list(P._records_py(batch, 61, len(recs), 100, recs[0][3]))
    assert [(x[2], x[3], x[4]) for x in native] == [(r[0], r[1], [tuple(h) for h in r[2]]) for r in recs]


def test_float32_vectors_use_float32_digits():
    """A Float32List (a local model's embedding row) is written with the shortest float32
    digits: json.dumps of the doubles those digits parse to, byte for byte, and every
    value parses back to the same float32."""
    import numpy as np
    from langstream_amd.utils.fastjson import Float32List, f32_rows
    rng = np.random.default_rng(3)
    for scale in (1e-30, 1e-6, 0.05, 1.0, 3e4, 1e15, 1e30):
        v = (rng.standard_normal(512) * scale).astype(np.float32)
        v[:6] = [0.0, -0.0, 1.0, -2.5, 1e-45, 123456790000000.0]
        got = fastjson.dumps({"e": Float32List(v.astype(np.float64).tolist()), "k": 1})
        want = jdumps({"e": [float(str(np.float32(x))) for x in v], "k": 1})
        assert got == want
        assert np.array_equal(np.array(json.loads(got)["e"], dtype=np.float32), v)
    rows = f32_rows(np.ones((2, 3), dtype=np.float32))
    assert [type(r) for r in rows] == [Float32List, Float32List] and rows[0] == [1.0, 1.0, 1.0]
    # anything but floats inside: the generic encoder, same bytes as json.dumps
    mixed = Float32List([1, 0.5, None])
    assert fastjson.dumps(mixed) == jdumps(mixed)
    # plain lists keep the double digits
    x = float(np.float32(0.1))
    assert fastjson.dumps([x]) == jdumps([x]) and fastjson.dumps(Float32List([x])) == "[0.1]"
    # user / EL code stored a double in a Float32List: no silent float32 rounding
    row = f32_rows(np.full((1, 4), 0.5, dtype=np.float32))[0]
    row[1] = 0.1                                    # not a float32 value
    row.append(1 / 3)
    assert fastjson.dumps(row) == jdumps(row) == "[0.5,0.1,0.5,0.5,0.3333333333333333]"
    assert fastjson.dumps(Float32List([float("nan"), 2.0])) == jdumps([float("nan"), 2.0])


def test_f32_matrix_matches_numpy():
    rng = random.Random(3)
    rows = [[rng.uniform(-2, 2) for _ in range(17)] for _ in range(5)]
    rows[2][3] = 7                                     # ints convert too
    got = fastjson.f32_matrix(rows)
    assert got.dtype == np.float32 and got.shape == (5, 17)
    np.testing.assert_array_equal(got, np.asarray(rows, dtype=np.float32))
    with pytest.raises(ValueError):
        fastjson.f32_matrix([[1.0, 2.0], [3.0]])       # ragged
    with pytest.raises((TypeError, ValueError)):
        fastjson.f32_matrix([[1.0, "x"]])              # non-numeric
