"""Configuration models, validator and documentation generator.

The reference annotates one Java class per agent / resource / asset type
(``@AgentConfig``/``@ConfigProperty``, ``langstream-api/.../api/doc/*``) and validates
application YAML against it reflectively (``CORE/impl/uti/ClassConfigValidator.java:148-583``);
``DocumentationGenerator.java`` turns the same classes into the ``/api/docs`` JSON.
Here the models are plain data (``Model`` / ``Prop``), one table for each kind, and the
same two consumers read them:

* ``validate_agent`` / ``validate_resource`` / ``validate_asset``: unknown keys are
  rejected (listing the known ones) unless the model allows them (python-* agents),
  required keys must be present, values must convert to the declared type (numbers and
  booleans may be given as strings, as Jackson's coercion allows), nested objects and
  list items are validated recursively, EL-typed properties must parse, and defaults are
  filled into the returned configuration.  Errors use the reference's wording:
  ``Found error on agent configuration (agent: 'n', type: 't'). Property 'k' is required``.
* ``generate_docs(version)``: ``{version, agents, resources, assets}`` with, per type,
  ``{type, name, description, properties: {key: {description, required, type,
  defaultValue, items?, properties?, extendedValidationType?}}}``.

MI355X-native additions are declared the same way (``local-gpu-configuration`` resource,
``local``/``local-gpu`` datasources, ``vector-collection`` asset, extra generation knobs
``seed``/``top-k``/``ignore-eos`` of the in-process engine).
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional


@dataclass
class Prop:
    type: str                                   # string | integer | number | boolean | array | object
    description: str = ""
    required: bool = False
    default: Any = None
    items: Optional["Prop"] = None
    properties: Optional[Dict[str, "Prop"]] = None
    el: bool = False                            # value is an EL expression (or a list of them)

    def doc(self) -> Dict[str, Any]:
        d: Dict[str, Any] = {"description": self.description, "required": self.required, "type": self.type}
        if self.default is not None:
            d["defaultValue"] = self.default
        if self.items is not None:
            d["items"] = self.items.doc()
        if self.properties is not None:
            d["properties"] = {k: v.doc() for k, v in self.properties.items()}
        if self.el:
            d["extendedValidationType"] = "EL_EXPRESSION"
        return d


@dataclass
class Model:
    name: str
    description: str
    properties: Dict[str, Prop] = field(default_factory=dict)
    allow_unknown: bool = False

    def doc(self, type_: str) -> Dict[str, Any]:
        return {"type": type_, "name": self.name, "description": self.description,
                "properties": {k: v.doc() for k, v in self.properties.items()}}


def S(desc="", required=False, default=None, el=False):
    return Prop("string", desc, required, default, el=el)


def I(desc="", required=False, default=None):
    return Prop("integer", desc, required, default)


def N(desc="", required=False, default=None):
    return Prop("number", desc, required, default)


def B(desc="", required=False, default=None):
    return Prop("boolean", desc, required, default)


def L(desc="", required=False, items=None, default=None, el=False):
    return Prop("array", desc, required, default, items=items, el=el)


def O(desc="", required=False, properties=None):
    return Prop("object", desc, required, properties=properties)


# ------------------------------------------------------------------ shared property groups
_COMPOSABLE = {"composable": B("Whether the planner may fuse this agent with its neighbours.", default=True),
               "when": S("EL condition; the step runs only for records where it is true.", el=True)}
_FIELD = O(properties={"name": S("Target field (value.x, key.x, properties.x, destinationTopic, ...).", True),
                       "expression": S("EL expression producing the field value.", True, el=True),
                       "type": S("Output type (STRING, INT32, INT64, FLOAT, DOUBLE, BOOLEAN, DATE, ...)."),
                       "optional": B("Whether a null result is allowed.", default=False)})
_NAMED_EXPR = O(properties={"name": S("Field name.", True), "expression": S("EL expression.", True, el=True)})
_GEN = {
    "model": S("Model name (the served model for local-gpu; a provider model id otherwise).", True),
    "stream-to-topic": S("Topic to stream partial completions to."),
    "stream-response-completion-field": S("Field of the streamed messages that holds the chunk."),
    "min-chunks-per-message": I("Tokens per streamed message at the start (doubles per message).", default=20),
    "completion-field": S("Field to write the completion to."),
    "stream": B("Stream tokens as they are generated.", default=True),
    "log-field": S("Field to write the request/response log to."),
    "max-tokens": I("Maximum number of generated tokens."),
    "temperature": N("Sampling temperature (0 = greedy)."),
    "top-p": N("Nucleus sampling mass."),
    "top-k": I("Top-k sampling cut (local-gpu engine)."),
    "seed": I("Sampling seed (local-gpu engine)."),
    "ignore-eos": B("Keep generating past end-of-sequence up to max-tokens (local-gpu engine)."),
    "logit-bias": O("Token id -> logit bias."),
    "user": S("End-user id forwarded to the provider."),
    "stop": L("Stop sequences.", items=S()),
    "presence-penalty": N("Presence penalty."),
    "frequency-penalty": N("Frequency penalty."),
    "ai-service": S("Id of the AI resource to use when several are configured."),
    "options": O("Provider-specific extra options."),
}

# ------------------------------------------------------------------ agents
AGENT_MODELS: Dict[str, Model] = {
    "drop-fields": Model("Drop fields", "Removes fields from the key or value of the record.", {
        "fields": L("Fields to drop.", True, S()), "part": S("key or value (default: both)."), **_COMPOSABLE}),
    "merge-key-value": Model("Merge key-value format", "Merges the key fields into the value.", {**_COMPOSABLE}),
    "unwrap-key-value": Model("Unwrap key-value format", "Replaces the record by its key or its value.", {
        "unwrapKey": B("Unwrap the key instead of the value.", default=False),
        "unwrap-key": B("Alias of unwrapKey (the transform-function spelling)."), **_COMPOSABLE}),
    "cast": Model("Cast record to another schema", "Converts key/value to another schema type.", {
        "schema-type": S("Target schema type (STRING, BYTES, INT32, ...).", True), "part": S("key or value."),
        **_COMPOSABLE}),
    "flatten": Model("Flatten record fields", "Flattens nested structures into delimited field names.", {
        "delimiter": S("Delimiter between path segments.", default="_"), "part": S("key or value."), **_COMPOSABLE}),
    "drop": Model("Drop the record", "Drops records (optionally only those matching 'when').", {**_COMPOSABLE}),
    "compute": Model("Compute values from the record", "Computes fields with EL expressions.", {
        "fields": L("Fields to compute.", True, _FIELD), **_COMPOSABLE}),
    "compute-ai-embeddings": Model("Compute embeddings of the record",
                                   "Embeds a templated text (batched on the GPU for local-gpu).", {
        "model": S("Embedding model.", default="text-embedding-ada-002"),
        "text": S("Mustache template of the text to embed.", True),
        "embeddings-field": S("Field to write the vector to.", True),
        "loop-over": S("EL list to embed one text per element of."),
        "batch-size": I("Records per embedding batch.", default=10),
        "concurrency": I("Batches in flight.", default=4),
        "flush-interval": I("Max ms a partial batch waits.", default=0),
        "ai-service": S("Id of the AI resource to use."), "options": O("Provider options."),
        "arguments": O("Provider arguments."), "model-url": S("Model URL (Hugging Face local models)."),
        **_COMPOSABLE}),
    "query": Model("Query", "Runs a query on a datasource and writes the results to a field.", {
        "query": S("Query text with ? placeholders.", True), "loop-over": S("EL list to run one query per element.",
                                                                            el=True),
        "fields": L("EL expressions bound to the ? placeholders.", items=S(), el=True),
        "output-field": S("Field to write the results to.", True),
        "only-first": B("Keep only the first row.", default=False), "datasource": S("Datasource resource id.", True),
        "mode": S("query or execute.", default="query"), "generated-keys": L("Keys to return for execute.",
                                                                             items=S()),
        **_COMPOSABLE}),
    "ai-chat-completions": Model("Compute chat completions", "Chat completion over templated messages.", {
        "messages": L("Messages (role + mustache content).", True,
                      O(properties={"role": S("system, user or assistant."),
                                    "content": S("Mustache template.", True)})), **_GEN, **_COMPOSABLE}),
    "ai-text-completions": Model("Compute text completions", "Text completion over a templated prompt.", {
        "prompt": L("Prompt lines (mustache).", True, S()), "logprobs-field": S("Field for token log-probs."),
        "logprobs": S("Number of log-probs to return."),
        "request-parameters": O("Extra request parameters."),
        "request-prompt-property": S("Request property carrying the prompt.", default="prompt"),
        "response-completions-expression": S("Expression extracting completions from the response."),
        **_GEN, **_COMPOSABLE}),
    "re-rank": Model("Re-rank", "Re-ranks a list of documents (MMR with BM25 + cosine).", {
        "field": S("Field holding the documents.", True), "output-field": S("Field to write the ranked list.", True),
        "algorithm": S("none or MMR.", default="none"), "query-embeddings": S("EL of the query vector."),
        "query-text": S("EL of the query text."), "embeddings-field": S("Per-document vector field."),
        "text-field": S("Per-document text field."), "max": I("Documents to keep.", default=100),
        "lambda": N("MMR relevance/diversity trade-off.", default=0.5), "k1": N("BM25 k1.", default=1.5),
        "b": N("BM25 b.", default=0.75)}),
    "flare-controller": Model("Flare Controller", "FLARE active retrieval: loops low-confidence generations.", {
        "tokens-field": S("Field with the generated tokens.", True),
        "logprobs-field": S("Field with the token log-probs.", True),
        "loop-topic": S("Topic to send records needing retrieval to.", True),
        "retrieve-documents-field": S("Field receiving the spans to retrieve for.", True),
        "min-prob": N("Probability below which a token triggers retrieval."),
        "min-token-gap": I("Tokens merged into one span."), "num-pad-tokens": I("Context tokens around a span."),
        "max-iterations": I("Loop limit."), "num-iterations-field": S("Field counting the iterations.")}),
    "text-extractor": Model("Text extractor", "Extracts plain text from PDF/HTML/Office documents.", {}),
    "language-detector": Model("Language detector", "Detects the text language into a property.", {
        "property": S("Property to write the language to.", default="language"),
        "allowedLanguages": L("Languages to keep (others are dropped).", items=S())}),
    "text-splitter": Model("Text splitter", "Splits text into chunks (recursive character splitter).", {
        "splitter_type": S("Splitter.", default="RecursiveCharacterTextSplitter"),
        "separators": L("Separators, tried in order.", items=S()),
        "keep_separator": B("Keep separators in chunks.", default=False),
        "chunk_size": I("Chunk size (in length_function units).", default=200),
        "chunk_overlap": I("Overlap between chunks.", default=100),
        "length_function": S("Length measure (cl100k_base tokens or length).", default="cl100k_base")}),
    "text-normaliser": Model("Text normaliser", "Lower-cases / trims text.", {
        "make-lowercase": B("Lower-case the text.", default=True), "trim-spaces": B("Trim spaces.", default=True)}),
    "document-to-json": Model("Document to JSON", "Wraps raw text into a JSON value.", {
        "text-field": S("Field for the text.", default="text"),
        "copy-properties": B("Copy record properties into the JSON.", default=True)}),
    "timer-source": Model("Timer source", "Emits a record every period-seconds.", {
        "fields": L("Fields of the emitted record.", items=_FIELD),
        "period-seconds": I("Period.", default=60)}),
    "log-event": Model("Log an event", "Logs records (fields or the whole record).", {
        "fields": L("Fields to log.", items=_NAMED_EXPR), "message": S("Message template."),
        "when": S("Condition.", default="true", el=True)}),
    "trigger-event": Model("Trigger event", "Emits an extra record to a destination topic.", {
        "fields": L("Fields of the new record.", items=_NAMED_EXPR), "when": S("Condition.", default="true", el=True),
        "continue-processing": B("Pass the original record on.", default=True),
        "destination": S("Destination topic.", True)}),
    "dispatch": Model("Dispatch agent", "Routes records to topics by condition.", {
        "routes": L("Routes.", items=O(properties={"when": S("Condition.", el=True), "destination": S("Topic."),
                                                   "action": S("dispatch or drop.", default="dispatch")}))}),
    "http-request": Model("Http Request", "Calls an HTTP endpoint per record.", {
        "url": S("URL template.", True), "output-field": S("Field for the response.", True),
        "method": S("HTTP method.", default="GET"), "headers": O("Header templates."),
        "query-string": O("Query-string templates."), "body": S("Body template."),
        "allow-redirects": B("Follow redirects.", default=True), "handle-cookies": B("Keep cookies.", default=True)}),
    "langserve-invoke": Model("Invoke LangServe", "Invokes a LangServe runnable (optionally streaming).", {
        "url": S("Endpoint URL.", True), "output-field": S("Field for the output.", True, default="value"),
        "content-field": S("Field of the streamed chunks.", default="content"),
        "stream-to-topic": S("Topic for streamed chunks."), "stream-response-field": S("Field of streamed messages."),
        "min-chunks-per-message": I("Chunks per streamed message at the start.", default=20),
        "debug": B("Log requests."), "method": S("HTTP method.", default="POST"), "headers": O("Headers."),
        "allow-redirects": B("Follow redirects.", default=True), "handle-cookies": B("Keep cookies.", default=True),
        "fields": L("Input fields.", items=_NAMED_EXPR)}),
    "webcrawler-source": Model("Web crawler source", "Crawls web sites, emitting one record per page.", {
        "state-storage": S("s3 or disk.", default="s3"), "bucketName": S("State bucket.", default="langstream-source"),
        "endpoint": S("S3 endpoint."), "access-key": S("S3 access key."), "secret-key": S("S3 secret key."),
        "region": S("S3 region."), "allowed-domains": L("Domain prefixes to crawl.", items=S()),
        "forbidden-paths": L("Path prefixes to skip.", items=S()), "max-urls": I("URL cap.", default=1000),
        "max-depth": I("Link depth cap.", default=50), "handle-robots-file": B("Honour robots.txt.", default=True),
        "scan-html-documents": B("Follow links in HTML.", default=True),
        "allow-non-html-contents": B("Emit non-HTML documents.", default=False),
        "seed-urls": L("Start URLs.", items=S()), "reindex-interval-seconds": I("Re-crawl interval."),
        "max-unflushed-pages": I("Pages between state flushes.", default=100),
        "min-time-between-requests": I("Politeness delay (ms).", default=500), "user-agent": S("User agent."),
        "max-error-count": I("Errors before a URL is given up.", default=5),
        "http-timeout": I("HTTP timeout (ms).", default=10000), "handle-cookies": B("Keep cookies.", default=True)}),
    "s3-source": Model("S3 Source", "Reads objects from an S3 bucket.", {
        "bucketName": S("Bucket.", default="langstream-source"), "endpoint": S("Endpoint."),
        "access-key": S("Access key."), "secret-key": S("Secret key."), "region": S("Region."),
        "idle-time": I("Seconds between scans.", default=5),
        "file-extensions": S("Comma-separated extensions to read.", default="pdf,docx,html,htm,md,txt")}),
    "azure-blob-storage-source": Model("Azure Blob Storage Source", "Reads blobs from an Azure container.", {
        "container": S("Container.", default="langstream-azure-source"), "endpoint": S("Endpoint.", True),
        "sas-token": S("SAS token."), "storage-account-name": S("Account name."),
        "storage-account-key": S("Account key."), "storage-account-connection-string": S("Connection string."),
        "idle-time": I("Seconds between scans.", default=5),
        "file-extensions": S("Comma-separated extensions to read.", default="pdf,docx,html,htm,md,txt")}),
    "camel-source": Model("Apache Camel Source", "Consumes a Camel component URI.", {
        "component-uri": S("Component URI.", True), "component-options": O("Component options."),
        "max-buffered-records": I("Buffer size.", default=100), "key-header": S("Header used as record key.")}),
    "identity": Model("Identity function", "Passes records through unchanged.", {}),
    "noop": Model("No-op", "Passes records through unchanged.", {}),
    "query-vector-db": Model("Query a vector database", "Runs a vector/DB query per record.", {
        "datasource": S("Datasource resource id.", True), "query": S("Query with ? placeholders.", True),
        "loop-over": S("EL list to run one query per element.", el=True),
        "fields": L("EL expressions bound to the ? placeholders.", items=S(), el=True),
        "output-field": S("Field to write the results to.", True),
        "only-first": B("Keep only the first row.", default=False), "mode": S("query or execute.", default="query"),
        "generated-keys": L("Keys returned by execute.", items=S()), **_COMPOSABLE}),
}
for _t, _d in (("python-source", "source"), ("python-processor", "processor"), ("python-function", "processor"),
               ("python-sink", "sink"), ("python-service", "service")):
    AGENT_MODELS[_t] = Model(f"Python custom {_d}", f"Runs a user Python {_d} from the application's python/ code.",
                             {"className": S("Fully qualified class name.", True)}, allow_unknown=True)
for _t in ("sink", "source"):
    AGENT_MODELS[_t] = Model(f"Kafka Connect {_t.capitalize()} agent", "Kafka Connect adapter (JVM only).",
                             {"connector.class": S("Connector class.", True)}, allow_unknown=True)

# vector-db-sink: the model depends on the datasource's service
_SINK_FIELDS = L("Fields to write.", True, _NAMED_EXPR)
VECTOR_SINK_MODELS: Dict[str, Model] = {
    "local": Model("Local GPU vector store", "Writes into the HBM-resident vector collection.", {
        "collection-name": S("Collection."), "fields": L("Fields to write.", items=_NAMED_EXPR),
        "batch-size": I("Max records per batched store mutation.", default=512)}),
    "jdbc": Model("JDBC", "Upserts rows into a table.", {
        "table-name": S("Table.", True), "fields": L("Columns.", True, O(properties={
            "name": S("Column.", True), "expression": S("EL expression.", True, el=True),
            "primary-key": B("Part of the primary key.", default=False)}))}),
    "cassandra": Model("Cassandra", "Writes rows with a column mapping.", {
        "table-name": S("Table.", True), "keyspace": S("Keyspace."),
        "mapping": S("col=expression, ... mapping.", True)}),
    "opensearch": Model("OpenSearch", "Indexes documents with the bulk API.", {
        "fields": _SINK_FIELDS, "id": S("EL of the document id."),
        "bulk-parameters": O("Bulk request parameters.", properties={
            "pipeline": S(), "refresh": S(), "require_alias": B(), "routing": S(), "timeout": S(),
            "wait_for_active_shards": S()}),
        "flush-interval": I("Max ms a partial batch waits.", default=1000),
        "batch-size": I("Documents per bulk request.", default=10)}),
    "solr": Model("Apache Solr", "Adds documents to a collection.", {
        "fields": _SINK_FIELDS, "commit-within": I("commitWithin (ms).", default=1000)}),
    "milvus": Model("Milvus", "Upserts entities into a collection.", {
        "fields": _SINK_FIELDS, "collection-name": S("Collection."), "database-name": S("Database."),
        "write-mode": S("upsert or insert.", default="upsert"), "primary-key": S("Primary key field.")}),
    "pinecone": Model("Pinecone", "Upserts vectors into an index.", {
        "vector.id": S("EL of the id."), "vector.vector": S("EL of the vector."),
        "vector.namespace": S("EL of the namespace."), "vector.metadata": O("Metadata field -> EL.")},
        allow_unknown=True),   # vector.metadata.<name> keys
    "astra-vector-db": Model("Astra Vector DB", "Upserts documents into a collection.", {
        "collection-name": S("Collection.", True), "fields": _SINK_FIELDS}),
}
for _a, _b in (("local-gpu", "local"), ("sqlite", "jdbc"), ("astra", "cassandra")):
    VECTOR_SINK_MODELS[_a] = VECTOR_SINK_MODELS[_b]
for _m in VECTOR_SINK_MODELS.values():
    _m.properties.setdefault("datasource", S("Datasource resource id.", True))

# ------------------------------------------------------------------ resources
RESOURCE_MODELS: Dict[str, Model] = {
    "open-ai-configuration": Model("OpenAI", "OpenAI or Azure OpenAI.", {
        "provider": S("openai or azure.", default="openai"), "access-key": S("API key.", True), "url": S("Azure URL.")}),
    "vertex-configuration": Model("Vertex AI", "Google Vertex AI.", {
        "url": S("Endpoint.", True), "region": S("Region.", True), "project": S("Project.", True),
        "token": S("Access token."), "serviceAccountJson": S("Service account JSON.")}),
    "hugging-face-configuration": Model("Hugging Face", "Hugging Face inference API or local models.", {
        "provider": S("api or local.", default="api"), "api-url": S("Inference URL."),
        "model-check-url": S("Model metadata URL."), "access-key": S("API token.")}),
    "ollama-configuration": Model("Ollama", "Ollama server.", {"url": S("Server URL.", True)}),
    "bedrock-configuration": Model("Amazon Bedrock", "Amazon Bedrock.", {
        "access-key": S("Access key.", True), "secret-key": S("Secret key.", True),
        "region": S("Region.", default="us-east-1"), "endpoint-override": S("Endpoint override.")}),
    "local-gpu-configuration": Model("Local GPU engine", "In-process MI355X engines (Llama decode + embeddings).", {
        "model": S("Chat/completion model config name."), "embeddings-model": S("Embedding model config name."),
        "checkpoint": S("Safetensors checkpoint directory."), "tp": I("Tensor-parallel degree."),
        "max-batch": I("Max concurrent sequences."), "max-seq-len": I("Max sequence length.")},
        allow_unknown=True),
}
DATASOURCE_MODELS: Dict[str, Model] = {
    "cassandra": Model("Cassandra", "Apache Cassandra over CQL.", {
        "contact-points": S("host[:port], ...", True), "loadBalancing-localDc": S("Local datacenter.", True),
        "port": I("Port.", default=9042), "username": S("User."), "password": S("Password."),
        "keyspace": S("Default keyspace."), "tls": B("Use TLS."), "consistency": S("Consistency level.")}),
    "astra": Model("Astra DB", "DataStax Astra over CQL.", {
        "secureBundle": S("Secure connect bundle."), "token": S("AstraCS token."), "database": S("Database name."),
        "database-id": S("Database id."), "clientId": S("Client id."), "secret": S("Client secret."),
        "username": S("User."), "password": S("Password."), "environment": S("Astra environment.", default="PROD"),
        "contact-points": S("host[:port], ..."), "port": I("Port."), "keyspace": S("Default keyspace.")}),
    "jdbc": Model("JDBC", "Relational database (SQLite-backed here).", {
        "driverClass": S("Driver class."), "url": S("JDBC URL.", True), "user": S("User."),
        "password": S("Password.")}, allow_unknown=True),
    "opensearch": Model("OpenSearch", "OpenSearch cluster.", {
        "https": B("Use HTTPS.", default=True), "host": S("Host.", True), "port": I("Port.", default=9200),
        "region": S("AWS region."), "username": S("User."), "password": S("Password."),
        "index-name": S("Index.", True)}),
    "pinecone": Model("Pinecone", "Pinecone index.", {
        "api-key": S("API key.", True), "environment": S("Environment.", True),
        "project-name": S("Project.", True), "index-name": S("Index.", True),
        "server-side-timeout-sec": I("Timeout.", default=10), "endpoint": S("Endpoint override.")}),
    "milvus": Model("Milvus", "Milvus / Zilliz.", {
        "user": S("User.", default="default"), "host": S("Host."), "password": S("Password."),
        "port": I("Port.", default=19530), "url": S("URL."), "token": S("Token.")}),
    "solr": Model("Apache Solr", "Solr collection.", {
        "protocol": S("http or https.", default="http"), "user": S("User."), "password": S("Password."),
        "host": S("Host."), "port": I("Port.", default=8983), "collection-name": S("Collection.")}),
    "astra-vector-db": Model("Astra Vector DB", "Astra Data API.", {
        "endpoint": S("API endpoint."), "token": S("Token."), "keyspace": S("Keyspace.")}),
    "local": Model("Local GPU vector store", "HBM-resident vector collections + SQLite tables.", {
        "path": S("SQLite path."), "persist-directory": S("Vector-store persistence directory (WAL + snapshots)."),
        "fsync": B("fsync every WAL append (default: flush to the OS only)."), "collection": S("Default collection."),
        "collection-name": S("Default collection."), "url": S("SQLite URL.")}, allow_unknown=True),
}
for _a, _b in (("local-gpu", "local"), ("sqlite", "jdbc")):
    DATASOURCE_MODELS[_a] = DATASOURCE_MODELS[_b]
for _m in DATASOURCE_MODELS.values():
    _m.properties.setdefault("service", S("Datasource service.", True))

# ------------------------------------------------------------------ assets
ASSET_MODELS: Dict[str, Model] = {
    "jdbc-table": Model("JDBC table", "A table created with SQL statements.", {
        "datasource": S("Datasource.", True), "table-name": S("Table.", True),
        "create-statements": L("CREATE statements.", True, S()), "delete-statements": L("DROP statements.", items=S())}),
    "cassandra-table": Model("Cassandra table", "A table created with CQL statements.", {
        "datasource": S("Datasource.", True), "table-name": S("Table.", True), "keyspace": S("Keyspace.", True),
        "create-statements": L("CQL statements.", True, S()), "delete-statements": L("CQL statements.", items=S())}),
    "cassandra-keyspace": Model("Cassandra keyspace", "A keyspace created with CQL statements.", {
        "datasource": S("Datasource.", True), "keyspace": S("Keyspace.", True),
        "create-statements": L("CQL statements.", True, S()), "delete-statements": L("CQL statements.", items=S())}),
    "astra-keyspace": Model("Astra keyspace", "An Astra keyspace.", {
        "datasource": S("Datasource.", True), "keyspace": S("Keyspace.", True)}),
    "opensearch-index": Model("OpenSearch index", "An index with optional settings / mappings.", {
        "datasource": S("Datasource.", True), "mappings": S("Mappings JSON."), "settings": S("Settings JSON.")}),
    "solr-collection": Model("Solr collection", "A collection created with collection/schema API calls.", {
        "datasource": S("Datasource.", True), "create-statements": L("API calls.", True, O(properties={
            "api": S("/api/collections or /schema.", True), "method": S("HTTP method.", default="POST"),
            "body": S("JSON body.")}))}),
    "milvus-collection": Model("Milvus collection", "A collection created with Milvus commands.", {
        "datasource": S("Datasource.", True), "collection-name": S("Collection.", True),
        "database-name": S("Database."), "create-statements": L("JSON commands.", True, S())}),
    "astra-collection": Model("Astra collection", "A Data API vector collection.", {
        "datasource": S("Datasource.", True), "collection-name": S("Collection.", True),
        "vector-dimension": I("Vector dimension.", True)}),
    "vector-collection": Model("GPU vector collection", "An HBM-resident vector collection.", {
        "datasource": S("Datasource."), "collection-name": S("Collection.", True),
        "dimension": I("Vector dimension."), "dimensions": I("Vector dimension (alias).")}, allow_unknown=True),
}


# ------------------------------------------------------------------ validation
def _err(ref: str, prop: Optional[str], msg: str) -> ValueError:
    return ValueError(f"Found error on {ref}. Property '{prop}' {msg}" if prop else f"Found error on {ref}. {msg}")


_TYPE_NAMES = {"string": "java.lang.String", "integer": "int", "number": "double", "boolean": "boolean",
               "array": "java.util.List", "object": "java.util.Map"}


def _convert(p: Prop, v: Any, ref: str, key: str) -> Any:
    bad = _err(ref, key, f"has a wrong data type. Expected type: {_TYPE_NAMES[p.type]}")
    if isinstance(v, str) and "{{" in v:          # unresolved placeholder: checked after resolution
        return v
    if p.type == "string":
        if isinstance(v, (dict, list)):
            raise bad
        return v
    if p.type == "integer":
        if isinstance(v, bool):
            raise bad
        if isinstance(v, int):
            return v
        if isinstance(v, float) and v.is_integer():
            return int(v)
        if isinstance(v, str):
            try:
                return int(v.strip())
            except ValueError:
                raise bad from None
        raise bad
    if p.type == "number":
        if isinstance(v, bool):
            raise bad
        if isinstance(v, (int, float)):
            return v
        if isinstance(v, str):
            try:
                return float(v.strip())
            except ValueError:
                raise bad from None
        raise bad
    if p.type == "boolean":
        if isinstance(v, bool):
            return v
        if isinstance(v, str) and v.strip().lower() in ("true", "false"):
            return v.strip().lower() == "true"
        raise bad
    if p.type == "array":
        if isinstance(v, (list, tuple, set)):
            return list(v)
        raise bad
    if p.type == "object":
        if isinstance(v, dict):
            return v
        raise bad
    return v


def _check_el(p: Prop, v: Any, ref: str, key: str) -> None:
    from ..agents.genai.el import compile_expression
    exprs = v if isinstance(v, list) else [v]
    for e in exprs:
        if e is None:
            raise _err(ref, key, "A null value is not allowed in a list of EL expressions")
        if not isinstance(e, str):
            continue
        src = e.strip()
        if src.startswith("${") and src.endswith("}"):
            src = src[2:-1]
        try:
            compile_expression(src)
        except Exception as ex:  # noqa: BLE001
            raise _err(ref, key, f"has an invalid EL expression '{e}': {ex}") from None


def _validate_props(ref: str, parent: Optional[str], value: Optional[Dict[str, Any]], props: Dict[str, Prop],
                    allow_unknown: bool, fill_defaults: bool) -> Dict[str, Any]:
    value = value or {}
    if not allow_unknown:
        for k in value:
            if k not in props:
                full = k if parent is None else f"{parent}.{k}"
                raise _err(ref, full, f"is unknown, you may want to try with some of {list(props)}")
    out = dict(value)
    for k, p in props.items():
        full = k if parent is None else f"{parent}.{k}"
        v = value.get(k)
        if v is None:
            if p.required:
                raise _err(ref, full, "is required")
            if fill_defaults and p.default is not None:
                out[k] = copy.deepcopy(p.default)
            continue
        v = _convert(p, v, ref, full)
        if p.properties is not None and isinstance(v, dict):
            v = _validate_props(ref, full, v, p.properties, False, False)
        if p.items is not None and isinstance(v, list):
            items = []
            for i, it in enumerate(v):
                it = _convert(p.items, it, ref, f"{full}[{i}]") if it is not None else it
                if p.items.properties is not None and isinstance(it, dict):
                    it = _validate_props(ref, full, it, p.items.properties, False, False)
                items.append(it)
            v = items
        if p.el:
            _check_el(p, v, ref, full)
        out[k] = v
    return out


def validate_model(ref: str, model: Model, cfg: Optional[Dict[str, Any]], fill_defaults: bool = False,
                   allow_unknown: Optional[bool] = None) -> Dict[str, Any]:
    return _validate_props(ref, None, cfg, model.properties,
                           model.allow_unknown if allow_unknown is None else allow_unknown, fill_defaults)


def agent_ref(name: Optional[str], type_: str) -> str:
    return f"agent configuration (agent: '{name}', type: '{type_}')"


def validate_agent(name: Optional[str], type_: str, cfg: Optional[Dict[str, Any]],
                   service: Optional[str] = None) -> Dict[str, Any]:
    """Validate an agent's configuration; returns it with converted values.  Types
    without a model (plugins registered at runtime) are accepted as they are."""
    model = AGENT_MODELS.get(type_)
    if type_ == "vector-db-sink":
        model = VECTOR_SINK_MODELS.get(service or "local")
    if model is None:
        return dict(cfg or {})
    return validate_model(agent_ref(name, type_), model, cfg)


def validate_resource(name: Optional[str], type_: str, cfg: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    ref = f"resource configuration (resource: '{name}', type: '{type_}')"
    if type_ in ("datasource", "vector-database"):
        model = DATASOURCE_MODELS.get((cfg or {}).get("service"))
    else:
        model = RESOURCE_MODELS.get(type_)
    if model is None:
        return dict(cfg or {})
    return validate_model(ref, model, cfg)


def validate_asset(name: Optional[str], type_: str, cfg: Optional[Dict[str, Any]]) -> Dict[str, Any]:
    model = ASSET_MODELS.get(type_)
    if model is None:
        return dict(cfg or {})
    return validate_model(f"asset configuration (asset: '{name}', type: '{type_}')", model, cfg)


# ------------------------------------------------------------------ documentation
def generate_docs(version: str = "") -> Dict[str, Any]:
    """``ApiConfigurationModel`` JSON (``DocumentationGenerator.java``)."""
    agents = {t: m.doc(t) for t, m in sorted(AGENT_MODELS.items())}
    for svc, m in sorted(VECTOR_SINK_MODELS.items()):
        agents[f"vector-db-sink_{svc}"] = dict(m.doc("vector-db-sink"), name=f"Vector DB sink ({m.name})")
    resources = {t: m.doc(t) for t, m in sorted(RESOURCE_MODELS.items())}
    for svc, m in sorted(DATASOURCE_MODELS.items()):
        resources[f"datasource_{svc}"] = m.doc("datasource")
        resources[f"vector-database_{svc}"] = m.doc("vector-database")
    assets = {t: m.doc(t) for t, m in sorted(ASSET_MODELS.items())}
    if not version:
        try:
            from .. import __version__ as version  # type: ignore
        except ImportError:
            version = "dev"
    return {"version": version, "agents": agents, "resources": resources, "assets": assets}


def docs_markdown(docs: Optional[Dict[str, Any]] = None) -> str:
    """Human-readable rendering of ``generate_docs`` (one table per type)."""
    docs = docs or generate_docs()
    out: List[str] = [f"# Configuration reference ({docs['version']})", ""]
    for section in ("agents", "resources", "assets"):
        out += [f"## {section.capitalize()}", ""]
        for key, m in docs[section].items():
            out += [f"### `{key}` - {m['name']}", "", m["description"], ""]
            if not m["properties"]:
                out += ["(no configuration)", ""]
                continue
            out += ["| property | type | required | default | description |", "|---|---|---|---|---|"]

            def rows(props, prefix=""):
                for k, p in props.items():
                    dv = p.get("defaultValue")
                    out.append(f"| `{prefix}{k}` | {p['type']} | {'yes' if p['required'] else ''} | "
                               f"{'' if dv is None else f'`{dv}`'} | {p['description']} |")
                    if p.get("properties"):
                        rows(p["properties"], f"{prefix}{k}.")
                    if (p.get("items") or {}).get("properties"):
                        rows(p["items"]["properties"], f"{prefix}{k}[].")
            rows(m["properties"])
            out.append("")
    return "\n".join(out)
