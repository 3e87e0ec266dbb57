"""The reference's ``ComputeFieldTest`` (``langstream-ai-agents/src/test/java/com/datastax/oss/
streaming/ai/model/ComputeFieldTest.java``): compute field names resolve to (name, scope)
and a bad name fails with the reference's message, also when the compute step is built."""
import pytest

from langstream_amd.agents.genai.steps import ComputeStep, compute_field_scope


def test_invalid_compute_field_name():
    msg = ("Invalid compute field name: newStringField. It should be prefixed with 'key.' or 'value.' or "
           "'properties.' or be one of [key, value, destinationTopic, messageKey]")
    with pytest.raises(ValueError) as e:
        compute_field_scope("newStringField")
    assert str(e.value) == msg
    with pytest.raises(ValueError) as e:
        ComputeStep({"fields": [{"name": "newStringField", "expression": "'Hotaru'", "type": "STRING"}]})
    assert str(e.value) == msg


@pytest.mark.parametrize("scoped,name,scope", [
    ("key.newStringField", "newStringField", "key"),          # testValidKeyComputeFieldName
    ("value.newStringField", "newStringField", "value"),      # testValidValueComputeFieldName
    ("destinationTopic", "destinationTopic", "header"),       # testValidHeaderComputeFieldName
    ("value", "value", "primitive"),                          # testPrimitiveValueComputeFieldName
    ("key", "key", "primitive"),                              # testPrimitiveKeyComputeFieldName
    ("properties.p1", "p1", "header.properties"),
])
def test_compute_field_scopes(scoped, name, scope):
    assert compute_field_scope(scoped) == (name, scope)
    ComputeStep({"fields": [{"name": scoped, "expression": "'Hotaru'", "type": "STRING"}]})
