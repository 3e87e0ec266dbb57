"""GenAI toolkit planning (CORE/agents/ai/GenAIToolKitFunctionAgentProvider.java:68-286).

The 11 step types (drop-fields ... ai-text-completions) become one runtime agent
``ai-tools`` whose configuration is ``{steps: [{type, ...}], <service-key>: resource
configuration, datasource: resource configuration}``.  The AI service is the resource
named by ``ai-service`` or else every AI resource present.  Service keys:
openai, huggingface, vertex, bedrock, ollama, and (MI355X-native, new) ``local`` for
``local-gpu-configuration`` -- the in-process GPU engines.
"""
from __future__ import annotations

import copy
from typing import Any, Dict

from ..api.model import AgentConfiguration, Application

AI_SERVICE_KEYS = {
    "open-ai-configuration": "openai",
    "hugging-face-configuration": "huggingface",
    "vertex-configuration": "vertex",
    "bedrock-configuration": "bedrock",
    "ollama-configuration": "ollama",
    "local-gpu-configuration": "local",
}
AI_STEPS = ("compute-ai-embeddings", "ai-chat-completions", "ai-text-completions")
DATASOURCE_STEPS = ("query",)


def resolve_datasource(resource_id: str, app: Application) -> Dict[str, Any]:
    r = app.resources.get(resource_id)
    if r is None:
        raise ValueError(f"Resource {resource_id} not found")
    if r.type not in ("datasource", "vector-database"):
        raise ValueError(f"Resource {resource_id} is not type=datasource")
    from .resources import resource_implementation
    return resource_implementation(r)


def build_genai_configuration(ac: AgentConfiguration, cfg: Dict[str, Any], app: Application) -> Dict[str, Any]:
    from .resources import resource_implementation
    step = copy.deepcopy(cfg)
    step["type"] = ac.type
    out: Dict[str, Any] = {}
    if ac.type in AI_STEPS:
        rid = step.pop("ai-service", None)
        if rid is not None:
            r = app.resources.get(rid)
            if r is None:
                raise ValueError(f"Resource {rid} not found")
            key = AI_SERVICE_KEYS.get(r.type)
            if key is None:
                raise ValueError(f"Resource {rid} is not in types: {sorted(AI_SERVICE_KEYS)}")
            out[key] = resource_implementation(r)
        else:
            found = False
            for r in app.resources.values():
                key = AI_SERVICE_KEYS.get(r.type)
                if key is not None:
                    out[key] = resource_implementation(r)
                    found = True
            if not found:
                raise ValueError(f"Found error on agent configuration (agent: '{ac.name or ac.id}', type: "
                                 f"'{ac.type}'). No ai service resource found in application configuration. "
                                 f"One of {', '.join(sorted(AI_SERVICE_KEYS))} must be defined.")
    if ac.type in DATASOURCE_STEPS:
        ds = step.pop("datasource", None)
        if ds is None:
            raise ValueError(f"Found error on agent configuration (agent: '{ac.name or ac.id}', type: 'query'). "
                             f"Property 'datasource' is required")
        out["datasource"] = resolve_datasource(ds, app) if isinstance(ds, str) else ds
    composable = step.get("composable", True)
    out["steps"] = [step]
    out["composable"] = composable
    return out
