"""Kafka client security: TLS and SASL/PLAIN (the Astra Streaming / Confluent Cloud shape
of the reference's ``examples/instances/astra.yaml``: ``security.protocol: SASL_SSL``,
``sasl.mechanism: PLAIN``, ``sasl.jaas.config: ... PlainLoginModule required
username='..' password='..';``).

``SecurityConfig.from_config`` reads the Java client property names from the streaming
cluster's ``admin`` map (consumer / producer maps may override):
  security.protocol              PLAINTEXT | SSL | SASL_PLAINTEXT | SASL_SSL
  sasl.mechanism                 PLAIN (the only mechanism implemented; others fail loudly)
  sasl.jaas.config               username / password are taken from it
  ssl.truststore.location        a PEM CA bundle (JKS stores are not readable here)
  ssl.truststore.certificates    inline PEM CA certificates
  ssl.endpoint.identification.algorithm   "" disables hostname verification (Java default: https)
  ssl.check.hostname / ssl.verify (extensions) false disables verification
The connection handshake: TCP -> TLS (SSL / SASL_SSL) -> SaslHandshake v1 (mechanism) ->
SaslAuthenticate v0 with the PLAIN message ``\\0username\\0password``.
"""
from __future__ import annotations

import re
import ssl
from dataclasses import dataclass
from typing import Any, Dict, Optional

_JAAS_KV = re.compile(r"""(\w+)\s*=\s*(?:'([^']*)'|"([^"]*)")""")


@dataclass
class SecurityConfig:
    protocol: str = "PLAINTEXT"
    mechanism: str = "PLAIN"
    username: Optional[str] = None
    password: Optional[str] = None
    cafile: Optional[str] = None
    cadata: Optional[str] = None
    check_hostname: bool = True
    verify: bool = True

    @property
    def tls(self) -> bool:
        return self.protocol in ("SSL", "SASL_SSL")

    @property
    def sasl(self) -> bool:
        return self.protocol in ("SASL_PLAINTEXT", "SASL_SSL")

    @staticmethod
    def from_config(*maps: Optional[Dict[str, Any]]) -> "SecurityConfig":
        cfg: Dict[str, Any] = {}
        for m in maps:
            cfg.update({k: v for k, v in (m or {}).items() if v is not None})
        proto = str(cfg.get("security.protocol", "PLAINTEXT")).upper()
        if proto not in ("PLAINTEXT", "SSL", "SASL_PLAINTEXT", "SASL_SSL"):
            raise ValueError(f"unsupported security.protocol {proto}")
        sc = SecurityConfig(protocol=proto, mechanism=str(cfg.get("sasl.mechanism", "PLAIN")).upper())
        jaas = cfg.get("sasl.jaas.config")
        if jaas:
            kv = {m.group(1): m.group(2) if m.group(2) is not None else m.group(3) for m in _JAAS_KV.finditer(jaas)}
            sc.username, sc.password = kv.get("username"), kv.get("password")
        sc.username = cfg.get("sasl.username", sc.username)
        sc.password = cfg.get("sasl.password", sc.password)
        if sc.sasl:
            if sc.mechanism != "PLAIN":
                raise ValueError(f"sasl.mechanism {sc.mechanism} is not supported (PLAIN only)")
            if sc.username is None or sc.password is None:
                raise ValueError("SASL/PLAIN needs username and password (sasl.jaas.config)")
        loc = cfg.get("ssl.truststore.location")
        if loc:
            if str(loc).lower().endswith((".jks", ".p12", ".pfx")):
                raise ValueError("ssl.truststore.location must be a PEM file here (JKS/PKCS12 stores are not "
                                 "readable); convert it with keytool/openssl")
            sc.cafile = str(loc)
        sc.cadata = cfg.get("ssl.truststore.certificates") or None
        eia = cfg.get("ssl.endpoint.identification.algorithm")
        if eia is not None and str(eia).strip() == "":
            sc.check_hostname = False
        if str(cfg.get("ssl.check.hostname", "true")).lower() == "false":
            sc.check_hostname = False
        if str(cfg.get("ssl.verify", "true")).lower() == "false":
            sc.verify = sc.check_hostname = False
        return sc

    def ssl_context(self) -> ssl.SSLContext:
        ctx = ssl.create_default_context(cafile=self.cafile, cadata=self.cadata)
        ctx.check_hostname = self.check_hostname
        if not self.verify:
            ctx.verify_mode = ssl.CERT_NONE
        return ctx

    def plain_token(self) -> bytes:
        return b"\0" + (self.username or "").encode() + b"\0" + (self.password or "").encode()


PLAINTEXT = SecurityConfig()
