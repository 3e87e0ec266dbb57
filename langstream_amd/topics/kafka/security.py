"""Kafka client security: TLS and SASL/PLAIN (the Astra Streaming / Confluent Cloud shape
of the reference's ``examples/instances/astra.yaml``: ``security.protocol: SASL_SSL``,
``sasl.mechanism: PLAIN``, ``sasl.jaas.config: ... PlainLoginModule required
username='..' password='..';``).

``SecurityConfig.from_config`` reads the Java client property names from the streaming
cluster's ``admin`` map (consumer / producer maps may override):
  security.protocol              PLAINTEXT | SSL | SASL_PLAINTEXT | SASL_SSL
  sasl.mechanism                 PLAIN | SCRAM-SHA-256 | SCRAM-SHA-512 (others fail loudly)
  sasl.jaas.config               username / password are taken from it
  ssl.truststore.location        a PEM CA bundle (JKS stores are not readable here)
  ssl.truststore.certificates    inline PEM CA certificates
  ssl.endpoint.identification.algorithm   "" disables hostname verification (Java default: https)
  ssl.check.hostname / ssl.verify (extensions) false disables verification
The connection handshake: TCP -> TLS (SSL / SASL_SSL) -> SaslHandshake v1 (mechanism) ->
SaslAuthenticate v0 with the PLAIN message ``\\0username\\0password``, or for SCRAM
(RFC 5802 / RFC 7677, what the reference's Kafka client does for ``sasl.mechanism:
SCRAM-SHA-*`` with ``ScramLoginModule``) two SaslAuthenticate round trips: client-first
-> server-first (nonce, salt, iterations), client-final with the proof -> server-final,
whose server signature is verified (a broker that does not know the password fails).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import os
import re
import ssl
from dataclasses import dataclass
from typing import Any, Dict, Optional, Tuple

SCRAM_MECHANISMS = {"SCRAM-SHA-256": "sha256", "SCRAM-SHA-512": "sha512"}

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
            if sc.mechanism != "PLAIN" and sc.mechanism not in SCRAM_MECHANISMS:
                raise ValueError(f"sasl.mechanism {sc.mechanism} is not supported "
                                 f"(PLAIN, {', '.join(SCRAM_MECHANISMS)})")
            if sc.username is None or sc.password is None:
                raise ValueError(f"SASL/{sc.mechanism} needs username and password (sasl.jaas.config)")
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


# ---------------------------------------------------------------------------- SCRAM
def _b64(b: bytes) -> str:
    return base64.b64encode(b).decode()


def _scram_name(name: str) -> str:
    return name.replace("=", "=3D").replace(",", "=2C")


def _attrs(msg: str) -> Dict[str, str]:
    out = {}
    for part in msg.split(","):
        if len(part) >= 2 and part[1] == "=":
            out[part[0]] = part[2:]
    return out


class ScramError(Exception):
    pass


class ScramClient:
    """Client side of one SCRAM-SHA-256/512 exchange (RFC 5802 section 3, RFC 7677)."""

    def __init__(self, mechanism: str, username: str, password: str, nonce: Optional[str] = None):
        self.hash = SCRAM_MECHANISMS[mechanism.upper()]
        self.username, self.password = username, password
        self.nonce = nonce or base64.b64encode(os.urandom(24)).decode().rstrip("=")
        self.first_bare = f"n={_scram_name(username)},r={self.nonce}"
        self._server_sig: Optional[bytes] = None

    def _hmac(self, key: bytes, msg: bytes) -> bytes:
        return hmac.new(key, msg, self.hash).digest()

    def first(self) -> bytes:
        return ("n,," + self.first_bare).encode()

    def final(self, server_first: bytes) -> bytes:
        sf = server_first.decode()
        a = _attrs(sf)
        if "e" in a:
            raise ScramError(f"server error: {a['e']}")
        nonce, salt, iters = a.get("r", ""), base64.b64decode(a.get("s", "")), int(a.get("i", "0"))
        if not nonce.startswith(self.nonce) or iters < 1:
            raise ScramError("server-first message does not extend the client nonce")
        salted = hashlib.pbkdf2_hmac(self.hash, self.password.encode(), salt, iters)
        client_key = self._hmac(salted, b"Client Key")
        stored = hashlib.new(self.hash, client_key).digest()
        without_proof = f"c=biws,r={nonce}"
        auth = f"{self.first_bare},{sf},{without_proof}".encode()
        sig = self._hmac(stored, auth)
        proof = bytes(x ^ y for x, y in zip(client_key, sig))
        self._server_sig = self._hmac(self._hmac(salted, b"Server Key"), auth)
        return f"{without_proof},p={_b64(proof)}".encode()

    def verify(self, server_final: bytes) -> None:
        a = _attrs(server_final.decode())
        if "e" in a:
            raise ScramError(f"server error: {a['e']}")
        if self._server_sig is None or not hmac.compare_digest(base64.b64decode(a.get("v", "")), self._server_sig):
            raise ScramError("server signature mismatch: the broker does not know this user's credentials")


class ScramServer:
    """Server side (the in-tree broker's SCRAM users): credentials are derived from the
    clear password once (salt, iterations), as a broker's SCRAM credential store holds."""

    def __init__(self, mechanism: str, users: Dict[str, str], iterations: int = 4096):
        self.hash = SCRAM_MECHANISMS[mechanism.upper()]
        self.creds: Dict[str, Tuple[bytes, int, bytes, bytes]] = {}
        for u, pw in users.items():
            salt = os.urandom(16)
            salted = hashlib.pbkdf2_hmac(self.hash, pw.encode(), salt, iterations)
            ck = hmac.new(salted, b"Client Key", self.hash).digest()
            self.creds[u] = (salt, iterations, hashlib.new(self.hash, ck).digest(),
                             hmac.new(salted, b"Server Key", self.hash).digest())
        self.state: Optional[Tuple[str, str, str, str]] = None   # (user, first_bare, server_first, nonce)

    def step(self, msg: bytes) -> Tuple[bytes, Optional[bool]]:
        """-> (reply, None while in progress / True authenticated / False rejected)."""
        m = msg.decode(errors="replace")
        if self.state is None:
            if not m.startswith("n,,"):
                return b"e=other-error", False
            bare = m[3:]
            a = _attrs(bare)
            user = a.get("n", "").replace("=2C", ",").replace("=3D", "=")
            if user not in self.creds:
                return b"e=unknown-user", False
            salt, iters, _, _ = self.creds[user]
            nonce = a.get("r", "") + base64.b64encode(os.urandom(18)).decode()
            sf = f"r={nonce},s={_b64(salt)},i={iters}"
            self.state = (user, bare, sf, nonce)
            return sf.encode(), None
        user, bare, sf, nonce = self.state
        a = _attrs(m)
        without_proof = m[: m.rfind(",p=")] if ",p=" in m else m
        _, _, stored, server_key = self.creds[user]
        if a.get("r") != nonce:
            return b"e=other-error", False
        auth = f"{bare},{sf},{without_proof}".encode()
        sig = hmac.new(stored, auth, self.hash).digest()
        proof = base64.b64decode(a.get("p", ""))
        client_key = bytes(x ^ y for x, y in zip(proof, sig))
        if len(proof) != len(sig) or not hmac.compare_digest(hashlib.new(self.hash, client_key).digest(), stored):
            return b"e=invalid-proof", False
        return ("v=" + _b64(hmac.new(server_key, auth, self.hash).digest())).encode(), True
