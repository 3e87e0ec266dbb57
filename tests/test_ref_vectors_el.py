"""The reference's own expression-language test vectors, ported.

Sources (inputs and expected outputs copied as data, each case cites its Java test):
* ``langstream-agents/langstream-ai-agents/src/test/java/com/datastax/oss/streaming/ai/
  jstl/predicate/JstlPredicateTest.java`` -- keyValuePredicates, primitivePredicates,
  primitiveKeyValuePredicates, testInvalidWhen;
* ``.../jstl/JstlFunctionsTest.java`` -- case / contains / concat / timestampAdd (millis,
  UTC and +02:00 providers) / toBigDecimal / cast / split / unpack / toJson / fromJson /
  filter;
* ``.../jstl/JstlEvaluatorTest.java`` -- functionExpressionProvider,
  methodInvocationExpressionProvider, testPrimitiveValue, testLength, testNowFunction,
  testTimestampAddFunctionsNow.

Representation mapping (not a semantic difference): Java ``Instant`` results are compared
as epoch milliseconds (the form ``fn:timestampAdd`` / ``fn:now`` return here);
``BigDecimal`` as ``decimal.Decimal``.  The records of the Java fixtures
(``Utils.createNestedAvroKeyValueRecord(2)``, ``createContextWithPrimitiveRecord``) are
rebuilt as MutableRecords with the same key / value objects, message key, topics and
properties.  Divergences these vectors found were fixed in ``el.py`` (compact
``toJson``, ``fromJson('')`` -> null, exact ``toBigDecimal(value, scale)`` and the
double path without a scale, month clamping, exact millisecond arithmetic, LocalTime
deltas)."""
import datetime as dt
import struct
from decimal import Decimal

import pytest

from langstream_amd.agents.genai import el
from langstream_amd.agents.genai.el import eval_expression, eval_predicate
from langstream_amd.agents.genai.mutable import MutableRecord


def _ms(iso: str) -> int:
    return (dt.datetime.fromisoformat(iso.replace("Z", "+00:00")) -
            dt.datetime(1970, 1, 1, tzinfo=dt.timezone.utc)) // dt.timedelta(milliseconds=1)


def _nested(levels: int = 2) -> dict:
    """Utils.createNestedAvroRecord(levels) as a map."""
    last = {f"level{levels}String": f"level{levels}_1", f"level{levels}Integer": 9, f"level{levels}Double": 8.8,
            f"level{levels}Array": [f"level{levels}_1", f"level{levels}_2"],
            f"level{levels}StringWithPropsAndAlias": f"level{levels}_WithProps",
            f"level{levels}Union": f"level{levels}_2", f"level{levels}Null": None, f"level{levels}NullRecord": None}
    rec = last
    for lv in range(levels - 1, 0, -1):
        rec = {f"level{lv}String": f"level{lv}_1", f"level{lv}Record": rec}
    return rec


def _kv_avro_record() -> MutableRecord:
    """Utils.createNestedAvroKeyValueRecord(2) through newTransformContext."""
    m = MutableRecord(key=_nested(2), value=_nested(2), properties={"p1": "v1", "p2": "v2"}, input_topic="topic-1",
                      event_time=1662493532)
    m.output_topic = "dest-topic-1"
    m.message_key = "key1"
    return m


def _primitive(value, message_key) -> MutableRecord:
    """Utils.createContextWithPrimitiveRecord(schema, value, key) for a non-KV schema: the
    record key is the message key."""
    m = MutableRecord(key=message_key, value=value)
    m.message_key = message_key
    return m


def _primitive_kv(k, v, message_key) -> MutableRecord:
    m = MutableRecord(key=k, value=v)
    m.message_key = message_key
    return m


# ------------------------------------------------------------------ JstlPredicateTest
KEY_VALUE_PREDICATES = [   # JstlPredicateTest.keyValuePredicates
    ("key.level1String == 'level1_1'", True),
    ("key.level1Record.level2String == 'level2_1'", True),
    ("key.level1Record.level2Integer == 9", True),
    ("key.level1Record.level2Double == 8.8", True),
    ("key.level1Record.level2Array[0] == 'level2_1'", True),
    ("value.level1Record.level2Integer > 8", True),
    ("value.level1Record.level2Double < 8.9", True),
    ("value.level1Record.level2Array[0] == 'level2_1'", True),
    ("messageKey == 'key1'", True),
    ("destinationTopic == 'dest-topic-1'", True),
    ("topicName == 'topic-1'", True),
    ("properties.p1 == 'v1'", True),
    ("properties.p2 == 'v2'", True),
    ("key.level1String == 'leVel1_1'", False),
    ("key.level1Record.random == 'level2_1'", False),
    ("key.level1Record.level2Integer != 9", False),
    ("key.level1Record.level2Double < 8.8", False),
    ("key.level1Record.level2Array[0] == 'non_existing_item'", False),
    ("key.randomKey == 'k1'", False),
    ("value.level1Record.level2Integer > 10", False),
    ("value.level1Record.level2Double < 0", False),
    ("value.randomValue < 0", False),
    ("messageKey == 'key2'", False),
    ("topicName != 'topic-1'", False),
    ("properties.p2 == 'v3'", False),
    ("randomHeader == 'h1'", False),
]


@pytest.mark.parametrize("when,match", KEY_VALUE_PREDICATES)
def test_predicate_key_value_avro(when, match):
    """JstlPredicateTest.testKeyValueAvro"""
    assert eval_predicate(when, _kv_avro_record().el_context()) is match


_STR = ("str", "test-message", "header-key")
_INT = ("int", 33, "header-key")
_KV = ("kv", ("key", 42), "header-key")
PRIMITIVE_PREDICATES = [   # JstlPredicateTest.primitivePredicates
    ("value=='test-message'", _STR, True),
    ("messageKey=='header-key'", _STR, True),
    ("key=='header-key'", _STR, True),
    ("value==33", _INT, True),
    ("value eq 33", _INT, True),
    ("value eq 32 + 1", _INT, True),
    ("value eq 34 - 1", _INT, True),
    ("value eq 66 / 2", _INT, True),
    ("value eq 66 div 2", _INT, True),
    ("value % 10 == 3", _INT, True),
    ("value mod 10 == 3", _INT, True),
    ("value>32", _INT, True),
    ("value gt 32", _INT, True),
    ("value<=33 && key=='header-key'", _INT, True),
    ("key=='key' && value==42", _KV, True),
    ("key=='key' and value==42", _KV, True),
    ("key=='key1' || value==42", _KV, True),
    ("key=='key1' or value==42", _KV, True),
    ("key=='key' && value==42", _KV, True),
    ("value=='test-message-'", _STR, False),
    ("key!='header-key'", _STR, False),
    ("key ne 'header-key'", _STR, False),
    ("value==34", _INT, False),
    ("value>33", _INT, False),
    ("value<=20 && key=='test-key'", _INT, False),
    ("value le 20 && key=='test-key'", _INT, False),
    # JstlPredicateTest.primitiveKeyValuePredicates (KV<String, Integer>, no message key)
    ("key=='key' && value==42", ("kv", ("key", 42), ""), True),
    ("key=='key' && value<42", ("kv", ("key", 42), ""), False),
]


def _ctx_of(spec) -> MutableRecord:
    kind, v, mk = spec
    return _primitive_kv(v[0], v[1], mk) if kind == "kv" else _primitive(v, mk)


@pytest.mark.parametrize("when,spec,match", PRIMITIVE_PREDICATES)
def test_predicate_primitive(when, spec, match):
    """JstlPredicateTest.testPrimitiveValueAvro / testPrimitiveKeyValueAvro"""
    assert eval_predicate(when, _ctx_of(spec).el_context()) is match


def test_predicate_invalid_when():
    """JstlPredicateTest.testInvalidWhen: a when that does not parse is rejected."""
    with pytest.raises(Exception):
        eval_predicate("`invalid", {})


# ------------------------------------------------------------------ JstlFunctionsTest
def _fn(name, *args):
    return el.FUNCTIONS[name](*args)


def test_functions_case_contains_concat():
    """JstlFunctionsTest.testUpperCase/LowerCase(+Integer/Null), testContains(+Integer/Null),
    testConcat(+Integer/Null)"""
    assert _fn("uppercase", "uppercase") == "UPPERCASE"
    assert _fn("uppercase", None) is None
    assert _fn("lowercase", "LOWERCASE") == "lowercase"
    assert _fn("uppercase", 10) == "10"
    for a, b in (("full text", "l t"), ("full text", "full"), ("full text", "text"), (123, "2"), ("123", 3),
                 (123, 3), ("123", "3")):
        assert _fn("contains", a, b) is True, (a, b)
    for a, b in (("full text", "lt"), ("full text", "fll"), ("full text", "txt"), (123, "4"), ("123", 4), (123, 4),
                 ("123", "4"), ("null", None), (None, "null"), (None, None)):
        assert _fn("contains", a, b) is False, (a, b)
    assert _fn("concat", "full ", "text") == "full text"
    assert _fn("concat", 1, 2) == "12" and _fn("concat", "1", 2) == "12" and _fn("concat", 1, "2") == "12"
    assert _fn("concat", None, "text") == "text" and _fn("concat", "full ", None) == "full "
    assert _fn("concat", None, None) == ""


_UNITS = [("years", "2027-10-02T01:02:03Z", "2019-10-02T01:02:03Z"),
          ("months", "2023-03-02T01:02:03Z", "2022-07-02T01:02:03Z"),
          ("days", "2022-10-07T01:02:03Z", "2022-09-29T01:02:03Z"),
          ("hours", "2022-10-02T06:02:03Z", "2022-10-01T22:02:03Z"),
          ("minutes", "2022-10-02T01:07:03Z", "2022-10-02T00:59:03Z"),
          ("seconds", "2022-10-02T01:02:08Z", "2022-10-02T01:02:00Z"),
          ("millis", "2022-10-02T01:02:03.005Z", "2022-10-02T01:02:02.997Z"),
          ("nanos", "2022-10-02T01:02:03.005Z", "2022-10-02T01:02:02.997Z")]
_BASE = "2022-10-02T01:02:03Z"
_TWO_H = 2 * 3600 * 1000


def _timestamp_cases():
    out = []
    for unit, plus5, minus3 in _UNITS:
        d5, d3 = (5_000_000, -3_000_000) if unit == "nanos" else (5, -3)
        for provider, inp, shift in (("millisTimestampAddProvider", _ms(_BASE), 0),
                                     ("utcTimestampAddProvider", _BASE, 0),
                                     ("nonUtcTimestampAddProvider", "2022-10-02T01:02:03+02:00", _TWO_H)):
            out += [(provider, inp, 0, unit, _ms(_BASE) - shift), (provider, inp, d5, unit, _ms(plus5) - shift),
                    (provider, inp, d3, unit, _ms(minus3) - shift)]
    return out


@pytest.mark.parametrize("provider,inp,delta,unit,expected", _timestamp_cases())
def test_timestamp_add(provider, inp, delta, unit, expected):
    """JstlFunctionsTest.testAddDateMillis / testAddDateUTC / testAddDateNonUTC"""
    assert _fn("timestampAdd", inp, delta, unit) == expected


def test_timestamp_add_conversions_and_errors():
    """JstlFunctionsTest.testAddDateDeltaConversion / testAddDateUnitConversion /
    testAddDateInvalidUnit / testInvalidAddDate"""
    assert _fn("timestampAdd", "2022-10-02T01:02:03Z", dt.time(1, 0, 0), "millis") == _ms("2022-10-02T02:02:03Z")
    assert _fn("timestampAdd", "2022-10-02T01:02:03Z", 1, b"hours") == _ms("2022-10-02T02:02:03Z")
    with pytest.raises(ValueError, match="Invalid unit: lightyear. Should be one of"):
        _fn("timestampAdd", 0, 0, "lightyear")
    with pytest.raises(ValueError):
        _fn("dateadd", True, 0, "days")


_BIG = Decimal("12.34567890123456789012345678901234567890")
TO_BIG_DECIMAL = [   # JstlFunctionsTest.toBigDecimalProvider
    ((1234567890123456789012345678901234567890).to_bytes(17, "big", signed=True), 38, _BIG),
    ("1234567890123456789012345678901234567890", "38", _BIG),
    (12345678, 4, Decimal("1234.5678")),
    (12345678, 4, Decimal("1234.5678")),
]
_F32 = struct.unpack("<f", struct.pack("<f", 1234.5678))[0]     # the Java float 1234.5678f
TO_BIG_DECIMAL_NO_SCALE = [   # JstlFunctionsTest.toBigDecimalWithoutScaleProvider (via a double)
    ("12.34567890123456789012345678901234567890", Decimal(repr(12.34567890123456789012345678901234567890))),
    (12.34567890123456789012345678901234567890, Decimal(repr(12.34567890123456789012345678901234567890))),
    (_F32, Decimal("1234.5677490234375")),
    (1234567, Decimal("1234567.0")),
    (1234567, Decimal("1234567.0")),
]


@pytest.mark.parametrize("value,scale,expected", TO_BIG_DECIMAL)
def test_to_big_decimal(value, scale, expected):
    """JstlFunctionsTest.testToBigDecimal"""
    got = _fn("toBigDecimal", value, scale)
    assert got == expected and str(got) == str(expected)


@pytest.mark.parametrize("value,expected", TO_BIG_DECIMAL_NO_SCALE)
def test_to_big_decimal_without_scale(value, expected):
    """JstlFunctionsTest.testToBigDecimalWithoutScale"""
    assert _fn("toBigDecimal", value) == expected


def test_cast_split_unpack():
    """JstlFunctionsTest.testCast / testSplit / testUnpack"""
    assert _fn("toDouble", "1.2") == 1.2 and _fn("toDouble", None) is None
    assert _fn("toInt", "1.2") == 1 and _fn("toInt", None) is None
    assert _fn("split", "1,2", ",") == ["1", "2"] and _fn("split", "", ",") == [] and _fn("split", None, ",") is None
    assert _fn("unpack", "1,2", "field1,field2") == {"field1": "1", "field2": "2"}
    assert _fn("unpack", "", "field1,field2") == {"field1": None, "field2": None}
    assert _fn("unpack", None, "field1,field2") is None
    assert _fn("unpack", "1,2", "field1,field2,field3") == {"field1": "1", "field2": "2", "field3": None}
    assert _fn("unpack", "1", "field1,field2") == {"field1": "1", "field2": None}
    assert _fn("unpack", _fn("split", "1:2", ":"), "field1,field2") == {"field1": "1", "field2": "2"}
    assert _fn("unpack", [1.0, 2.0], "field1,field2") == {"field1": 1.0, "field2": 2.0}


def test_to_json_from_json():
    """JstlFunctionsTest.testToJson / testFromJson (Jackson's compact output)"""
    assert _fn("toJson", {"field1": 1}) == '{"field1":1}'
    assert _fn("toJson", None) == "null"
    assert _fn("toJson", "") == '""'
    assert _fn("toJson", [1, 2, 3]) == "[1,2,3]"
    assert _fn("fromJson", '{"field1":1}') == {"field1": 1}
    assert _fn("fromJson", None) is None and _fn("fromJson", "null") is None and _fn("fromJson", "") is None
    assert _fn("fromJson", '""') == "" and _fn("fromJson", "[1,2,3]") == [1, 2, 3]


_QUERY_RESULT = [{"name": "product1", "price": "1.2", "similarity": "0.9"},
                 {"name": "product2", "price": "1.7", "similarity": "0.1"}]


@pytest.mark.parametrize("expr,names", [
    ("fn:toDouble(record.similarity) >= 0.5", ["product1"]),
    ("fn:toDouble(record.similarity) < 0.5", ["product2"]),
    ("false", []),
    ("true", ["product1", "product2"]),
])
def test_filter_query_results(expr, names):
    """JstlFunctionsTest.testFilterQueryResults"""
    got = eval_expression(f"fn:filter(value.r, '{expr}')", {"value": {"r": _QUERY_RESULT}})
    assert [g["name"] for g in got] == names


@pytest.mark.parametrize("expr,names", [
    ("fn:toDouble(record.similarity) >= value.threshold", ["product1"]),
    ("fn:toDouble(record.similarity) < value.threshold", ["product2"]),
    ("false", []),
    ("true", ["product1", "product2"]),
])
def test_filter_query_results_with_context(expr, names):
    """JstlFunctionsTest.testFilterQueryResultsWithContext: the record's value is visible
    inside the filter expression"""
    m = MutableRecord(value={"threshold": "0.5", "r": _QUERY_RESULT})
    got = eval_expression(f"fn:filter(value.r, '{expr}')", m.el_context())
    assert [g["name"] for g in got] == names


# ------------------------------------------------------------------ JstlEvaluatorTest
_BYTES = b"Test-Message "
_MILLIS = _ms("2017-01-02T00:01:02Z")
FUNCTION_EXPRESSIONS = [   # JstlEvaluatorTest.functionExpressionProvider
    ("fn:uppercase('test')", _BYTES, "TEST"),
    ("fn:uppercase(value) == 'TEST-MESSAGE '", _BYTES, True),
    ("fn:uppercase(null)", _BYTES, None),
    ("fn:lowercase('TEST')", _BYTES, "test"),
    ("fn:lowercase(value) == 'test-message '", _BYTES, True),
    ("fn:lowercase(null)", _BYTES, None),
    ("fn:coalesce(null, 'another-value')", _BYTES, "another-value"),
    ("fn:coalesce('value', 'another-value')", _BYTES, "value"),
    ("fn:coalesce(fn:str(value), 'another-value')", _BYTES, "Test-Message "),
    ("fn:contains(value, 'Test')", _BYTES, True),
    ("fn:contains(value, 'random')", _BYTES, False),
    ("fn:contains(null, 'random')", _BYTES, False),
    ("fn:contains(value, null)", _BYTES, False),
    ("fn:trim('    trimmed      ')", _BYTES, "trimmed"),
    ("fn:trim(value)", _BYTES, "Test-Message"),
    ("fn:trim(null)", _BYTES, None),
    ("fn:concat(value, 'suffix')", _BYTES, "Test-Message suffix"),
    ("fn:concat(value, null)", _BYTES, "Test-Message "),
    ("fn:concat(null, 'suffix')", _BYTES, "suffix"),
    ("fn:concat('prefix-', value)", _BYTES, "prefix-Test-Message "),
    ("fn:replace(value, '.*-', '')", _BYTES, "Message "),
    ("fn:replace('Test-Message test', value, '')", _BYTES, "test"),
    ("fn:replace('Something test', '.* ', value)", _BYTES, "Test-Message test"),
    ("fn:replace(null, '.* ', '')", _BYTES, None),
    ("fn:replace('test', null, '')", _BYTES, "test"),
    ("fn:replace('test', '.*', null)", _BYTES, "test"),
    ("fn:timestampAdd('2017-01-02T00:01:02Z', 1, 'years')", _BYTES, _ms("2018-01-02T00:01:02Z")),
    ("fn:timestampAdd('2017-01-02T00:01:02Z', -1, 'months')", _BYTES, _ms("2016-12-02T00:01:02Z")),
    ("fn:timestampAdd('2017-01-02T00:01:02Z', 1, 'days')", _BYTES, _ms("2017-01-03T00:01:02Z")),
    ("fn:timestampAdd('2017-01-02T00:01:02Z', -1, 'hours')", _BYTES, _ms("2017-01-01T23:01:02Z")),
    ("fn:timestampAdd('2017-01-02T00:01:02Z', 1, 'minutes')", _BYTES, _ms("2017-01-02T00:02:02Z")),
    ("fn:timestampAdd('2017-01-02T00:01:02Z', -1, 'seconds')", _BYTES, _ms("2017-01-02T00:01:01Z")),
    ("fn:timestampAdd('2017-01-02T00:01:02Z', 1, 'millis')", _BYTES, _ms("2017-01-02T00:01:02.001Z")),
    ("fn:timestampAdd('2017-01-02T00:01:02Z', 1000000, 'nanos')", _BYTES, _ms("2017-01-02T00:01:02.001Z")),
    (f"fn:timestampAdd({_MILLIS}, 1, 'years')", _BYTES, _ms("2018-01-02T00:01:02Z")),
    (f"fn:timestampAdd({_MILLIS}, -1, 'months')", _BYTES, _ms("2016-12-02T00:01:02Z")),
    (f"fn:timestampAdd({_MILLIS}, 1, 'days')", _BYTES, _ms("2017-01-03T00:01:02Z")),
    (f"fn:timestampAdd({_MILLIS}, -1, 'hours')", _BYTES, _ms("2017-01-01T23:01:02Z")),
    (f"fn:timestampAdd({_MILLIS}, 1, 'minutes')", _BYTES, _ms("2017-01-02T00:02:02Z")),
    (f"fn:timestampAdd({_MILLIS}, -1, 'seconds')", _BYTES, _ms("2017-01-02T00:01:01Z")),
    (f"fn:timestampAdd({_MILLIS}, 1, 'millis')", _BYTES, _ms("2017-01-02T00:01:02.001Z")),
    (f"fn:timestampAdd({_MILLIS}, 1000000, 'nanos')", _BYTES, _ms("2017-01-02T00:01:02.001Z")),
    ("fn:timestampAdd(value, '1', 'millis')", dt.datetime(2017, 1, 2, 0, 1, 2, tzinfo=dt.timezone.utc),
     _ms("2017-01-02T00:01:02.001Z")),
    ("fn:timestampAdd('2017-01-02T00:01:02Z', 1, value)", b"millis", _ms("2017-01-02T00:01:02.001Z")),
]


@pytest.mark.parametrize("expr,value,expected", FUNCTION_EXPRESSIONS)
def test_evaluator_functions(expr, value, expected):
    """JstlEvaluatorTest.testFunctions"""
    assert eval_expression(expr, _primitive(value, "").el_context()) == expected


@pytest.mark.parametrize("expr", [   # JstlEvaluatorTest.methodInvocationExpressionProvider
    "value.contains('test')", "value.toUpperCase() == 'TEST-MESSAGE'",
    "value.toUpperCase().toLowerCase() == 'test-message'", "value.substring(0, 4) == 'test'",
    "value.contains('random')"])
def test_evaluator_method_invocations_disabled(expr):
    """JstlEvaluatorTest.testMethodInvocationsDisabled: no Java-style method calls"""
    with pytest.raises(Exception):
        eval_expression(expr, _primitive("test-message", "header-key").el_context())


def test_evaluator_primitive_length_now(monkeypatch):
    """JstlEvaluatorTest.testPrimitiveValue / testLength / testNowFunction /
    testTimestampAddFunctionsNow (a fixed clock)"""
    ctx = _primitive("test-message", "").el_context()
    assert eval_expression("value", ctx) == "test-message"
    assert str(eval_expression("fn:length(value)", ctx)) == "12"
    monkeypatch.setattr(el.time, "time", lambda: 0.123)
    assert eval_expression("fn:now()", ctx) == 123
    monkeypatch.setattr(el.time, "time", lambda: 5.0)
    assert eval_expression("fn:timestampAdd(fn:now(), -3333, 'seconds')", ctx) == 5000 - 3333 * 1000
