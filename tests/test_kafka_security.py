"""Kafka adapter: SASL/PLAIN over TLS with the reference's examples/instances/astra.yaml
configuration shape, and compressed record batches (gzip / snappy / lz4) on fetch and
produce.  The broker is the in-tree Kafka-protocol broker with a TLS listener (a
self-signed certificate made with the openssl CLI) that requires SASL/PLAIN."""
import shutil
import ssl
import subprocess
import time

import pytest

from langstream_amd.api.model import StreamingCluster
from langstream_amd.api.record import SimpleRecord
from langstream_amd.api.topics import TopicOffsetPosition
from langstream_amd.topics.kafka import KafkaTopicConnectionsRuntime, codecs
from langstream_amd.topics.kafka import protocol as P
from langstream_amd.topics.kafka.broker import KafkaBroker
from langstream_amd.topics.kafka.client import KafkaClient, KafkaError
from langstream_amd.topics.kafka.security import SecurityConfig


@pytest.fixture(scope="module")
def tls_broker(tmp_path_factory):
    if shutil.which("openssl") is None:
        pytest.skip("openssl CLI not available")
    d = tmp_path_factory.mktemp("tls")
    key, crt = d / "key.pem", d / "cert.pem"
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", str(key), "-out",
                    str(crt), "-days", "2", "-subj", "/CN=127.0.0.1", "-addext", "subjectAltName=IP:127.0.0.1"],
                   check=True, capture_output=True)
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(str(crt), str(key))
    b = KafkaBroker(ssl_context=ctx, sasl_users={"tenant-user": "s3cret"}).start()
    yield b, str(crt)
    b.stop()


def _astra_instance(bootstrap, cafile, user="tenant-user", password="s3cret"):
    # examples/instances/astra.yaml, resolved, + the CA of the test broker
    return StreamingCluster("kafka", {"admin": {
        "bootstrap.servers": bootstrap, "security.protocol": "SASL_SSL",
        "sasl.jaas.config": f"org.apache.kafka.common.security.plain.PlainLoginModule required "
                            f"username='{user}' password='{password}';",
        "sasl.mechanism": "PLAIN", "session.timeout.ms": "45000", "ssl.truststore.location": cafile}})


def test_sasl_ssl_roundtrip_astra_shape(tls_broker):
    broker, ca = tls_broker
    rt = KafkaTopicConnectionsRuntime()
    rt.init(_astra_instance(broker.bootstrap, ca))
    assert rt.security.tls and rt.security.sasl and rt.security.username == "tenant-user"
    prod = rt.create_producer("a", None, {"topic": "secure"})
    prod.write(SimpleRecord.of("k1", "hello over SASL_SSL")).result(10)
    rd = rt.create_reader(None, {"topic": "secure"}, TopicOffsetPosition.EARLIEST)
    rd.start()
    got = []
    deadline = time.time() + 10
    while not got and time.time() < deadline:
        got = rd.read().records
    assert [(r.key(), r.value()) for r in got] == [("k1", "hello over SASL_SSL")]
    rd.close()
    prod.close()


def test_sasl_wrong_password_rejected(tls_broker):
    broker, ca = tls_broker
    sc = SecurityConfig.from_config(_astra_instance(broker.bootstrap, ca, password="nope").configuration["admin"])
    with pytest.raises(KafkaError):
        KafkaClient(broker.bootstrap, security=sc).refresh_metadata()


def test_plaintext_client_cannot_talk_to_tls_listener(tls_broker):
    broker, _ = tls_broker
    with pytest.raises((ConnectionError, OSError)):
        KafkaClient(broker.bootstrap).refresh_metadata()


def test_security_config_validation():
    with pytest.raises(ValueError):
        SecurityConfig.from_config({"security.protocol": "SASL_SSL", "sasl.mechanism": "GSSAPI",
                                    "sasl.jaas.config": "x required username='a' password='b';"})
    sc = SecurityConfig.from_config({"security.protocol": "SASL_SSL", "sasl.mechanism": "SCRAM-SHA-512",
                                     "sasl.jaas.config": "x required username='a' password='b';"})
    assert sc.mechanism == "SCRAM-SHA-512" and sc.username == "a"
    with pytest.raises(ValueError):
        SecurityConfig.from_config({"security.protocol": "SASL_PLAINTEXT"})      # no credentials
    sc = SecurityConfig.from_config({"security.protocol": "SSL", "ssl.endpoint.identification.algorithm": ""})
    assert sc.tls and not sc.sasl and not sc.check_hostname


@pytest.mark.parametrize("codec", ["gzip", "snappy", "lz4"])
def test_compressed_batches_fetch_and_produce(codec):
    broker = KafkaBroker().start()
    try:
        rt = KafkaTopicConnectionsRuntime()
        rt.init(StreamingCluster("kafka", {"admin": {"bootstrap.servers": broker.bootstrap},
                                           "producer": {"compression.type": codec}}))
        prod = rt.create_producer("a", None, {"topic": "z"})
        for i in range(20):
            prod.write(SimpleRecord.of(f"k{i}", "payload " * (i + 1))).result(10)
        rd = rt.create_reader(None, {"topic": "z"}, TopicOffsetPosition.EARLIEST)
        rd.start()
        got = []
        deadline = time.time() + 10
        while len(got) < 20 and time.time() < deadline:
            got += rd.read().records
        assert [r.value() for r in got] == ["payload " * (i + 1) for i in range(20)]
        rd.close()
        prod.close()
    finally:
        broker.stop()


def test_codec_decoders_on_streams_with_back_references():
    import gzip
    # snappy: literal "abcd" + copy(offset 4, len 8)
    assert codecs.snappy_raw_decompress(bytes([12, 0x0C]) + b"abcd" + bytes([0x11, 0x04])) == b"abcdabcdabcd"
    # lz4 block: token(lit 4, match 4+4) "abcd" off 4, then a literal-only tail
    out = bytearray()
    codecs.lz4_block_decompress(bytes([0x44]) + b"abcd" + bytes([4, 0, 0x50]) + b"xyzwv", out)
    assert bytes(out) == b"abcdabcdabcdxyzwv"
    # gzip from the standard library encoder
    assert codecs.gzip_decompress(gzip.compress(b"hello" * 100)) == b"hello" * 100
    with pytest.raises(ValueError):
        codecs.decompress(codecs.ZSTD, b"\x28\xb5\x2f\xfd")
    # a batch compressed by a producer decodes through decode_batches
    recs = [(b"k", b"v" * 100, [], 5)]
    assert [x[3] for x in P.decode_batches(P.encode_batch(0, recs, codecs.GZIP), verify_crc=True)] == [b"v" * 100]


def test_scram_sha256_rfc7677_test_vector():
    """RFC 7677 section 3: user 'user', password 'pencil'."""
    from langstream_amd.topics.kafka.security import ScramClient
    c = ScramClient("SCRAM-SHA-256", "user", "pencil", nonce="rOprNGfwEbeRWgbNEkqO")
    assert c.first() == b"n,,n=user,r=rOprNGfwEbeRWgbNEkqO"
    sf = b"r=rOprNGfwEbeRWgbNEkqO%hvYDpWUa2RaTCAfuxFIlj)hNlF$k0,s=W22ZaJ0SNY7soEsUEjb6gQ==,i=4096"
    assert c.final(sf) == (b"c=biws,r=rOprNGfwEbeRWgbNEkqO%hvYDpWUa2RaTCAfuxFIlj)hNlF$k0,"
                           b"p=dHzbZapWIk4jUhN+Ute9ytag9zjfMHgsqmmiz7AndVQ=")
    c.verify(b"v=6rriTRBi23WpRR/wtup+mMhUZUn/dB5nLTJRsjl95G4=")


@pytest.mark.parametrize("mech", ["SCRAM-SHA-256", "SCRAM-SHA-512"])
def test_sasl_scram_roundtrip_and_rejection(tls_broker, mech):
    broker, ca = tls_broker
    inst = _astra_instance(broker.bootstrap, ca)
    inst.configuration["admin"]["sasl.mechanism"] = mech
    inst.configuration["admin"]["sasl.jaas.config"] = (
        "org.apache.kafka.common.security.scram.ScramLoginModule required username='tenant-user' password='s3cret';")
    rt = KafkaTopicConnectionsRuntime()
    rt.init(inst)
    prod = rt.create_producer("a", None, {"topic": "scram-" + mech[-3:]})
    prod.write(SimpleRecord.of("k", "via " + mech)).result(10)
    prod.close()
    bad = SecurityConfig.from_config({**inst.configuration["admin"], "sasl.jaas.config":
                                      "x required username='tenant-user' password='wrong';"})
    with pytest.raises(KafkaError):
        KafkaClient(broker.bootstrap, security=bad).refresh_metadata()
    nouser = SecurityConfig.from_config({**inst.configuration["admin"], "sasl.jaas.config":
                                         "x required username='ghost' password='s3cret';"})
    with pytest.raises(KafkaError):
        KafkaClient(broker.bootstrap, security=nouser).refresh_metadata()
