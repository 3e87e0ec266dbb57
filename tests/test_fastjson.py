"""Native JSON encoder (native/jsonenc.cpp) is byte-identical to json.dumps."""
import collections
import json
import random
import struct

import numpy as np
import pytest

from langstream_amd.utils import fastjson


def test_floats_match_repr():
    rnd = random.Random(7)
    vals = [0.0, -0.0, 1.0, -1.0, 1e16, 1e15, 1.5e16, 1e-5, 1e-4, 1.234e-4, 123.0, 1e22, 5e-324,
            1.7976931348623157e308, float("nan"), float("inf"), -float("inf"), 0.1, 9999999999999998.0]
    for _ in range(20000):
        vals.append(rnd.uniform(-1, 1) * 10 ** rnd.randint(-30, 30))
        vals.append(float(np.float32(rnd.gauss(0, 1))))
        vals.append(struct.unpack("d", struct.pack("Q", rnd.getrandbits(64)))[0])
    assert [fastjson.dumps(v) for v in vals] == [json.dumps(v) for v in vals]


def test_structures_and_strings():
    objs = [{"a": [1, 2, {"b": None, "c": True}], "é": "ünï \U0001f600\x7f\x00\"\\\n\t\r\b\f", 3: 4, 2.5: 1,
             None: 0, False: 1},
            [], {}, (1, 2), [10 ** 30, -10 ** 30, -5, 0], "x" * 1000, {"k": [[[]]]}, "汉字",
            {"embeddings": np.random.default_rng(0).standard_normal(384).astype(np.float32).tolist()}]
    for o in objs:
        assert fastjson.dumps(o) == json.dumps(o)
    assert fastjson.dumps(collections.OrderedDict(a=1, b=[1.5])) == json.dumps(collections.OrderedDict(a=1, b=[1.5]))


def test_unsupported_falls_back_to_json_errors():
    class Foo:
        pass
    with pytest.raises(TypeError):
        fastjson.dumps({"a": Foo()})
    cyc = []
    cyc.append(cyc)
    with pytest.raises(ValueError):
        fastjson.dumps(cyc)
