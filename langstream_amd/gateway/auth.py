"""Gateway authentication providers (``API/gateway/*``).

``authenticate(ctx) -> AuthResult(authenticated, reason, principal_values)``.

* ``http``   (``HttpAuthenticationProvider.java``): GET ``base-url + path-template``
  (``{tenant}`` substituted) with ``Authorization: Bearer <credentials>`` plus
  configured ``headers``; success iff the status is in ``accepted-statuses``
  (200, 201).  No principal values.
* ``jwt``    (``JwtAuthenticationProvider.java``): HS256/384/512 with ``secret-key`` or
  RS256/384/512 with ``public-key`` (PEM) or a JWKS fetched from ``jwks-uri`` or from
  the token's ``jku`` (followed only when its host matches a non-empty
  ``jwks-hosts-allowlist``); any other ``alg`` is rejected; ``exp``/``nbf`` checked;
  optional ``audience`` checked against ``audience-claim`` (aud); principal values are
  the string claims, ``subject`` = ``auth-claim`` (sub).  RSA verification is done with
  plain modular exponentiation (no crypto library is available offline).
* ``github`` (``GitHubAuthenticationProvider.java``): GET https://api.github.com/user with
  the token; principal values ``login``, ``id``, ``name``, ``email``.
* ``google`` (``GoogleAuthenticationProvider.java``): Google ID token = RS256 JWT whose
  ``aud`` must equal ``clientId``, verified against Google's JWKS; principal values
  ``subject``, ``email``, ``name``, ``locale``.
* test mode (``test-credentials`` + ``allow-test-mode``): principal values derived from
  sha256(credentials) exactly like ``GatewayRequestHandler.getPrincipalValues``.
"""
from __future__ import annotations

import base64
import re
import hashlib
import hmac
import json
import threading
import time
import urllib.parse
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional


@dataclass
class AuthResult:
    authenticated: bool
    reason: Optional[str] = None
    principal_values: Dict[str, str] = field(default_factory=dict)


def _cfg(c: Dict[str, Any], *names, default=None):
    for n in names:
        if c.get(n) is not None:
            return c[n]
    return default


def _b64url(s: str) -> bytes:
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def java_string_hash(s: str) -> int:
    h = 0
    for ch in s:
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= 1 << 31 else h


def test_principal_values(credentials: str) -> Dict[str, str]:
    subject = hashlib.sha256((credentials or "").encode()).hexdigest()
    return {"subject": subject, "email": f"{subject}@locahost", "name": subject, "login": subject,
            "id": str(java_string_hash(subject))}


# ---------------------------------------------------------------- RSA (PKCS#1 v1.5) verify
_DIGEST_INFO = {
    "SHA256": bytes.fromhex("3031300d060960864801650304020105000420"),
    "SHA384": bytes.fromhex("3041300d060960864801650304020205000430"),
    "SHA512": bytes.fromhex("3051300d060960864801650304020305000440"),
}


def rsa_pkcs1_verify(n: int, e: int, msg: bytes, sig: bytes, hash_name: str) -> bool:
    k = (n.bit_length() + 7) // 8
    if len(sig) != k:
        return False
    m = pow(int.from_bytes(sig, "big"), e, n).to_bytes(k, "big")
    digest = hashlib.new(hash_name.lower(), msg).digest()
    t = _DIGEST_INFO[hash_name] + digest
    expected = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
    return hmac.compare_digest(m, expected)


def _der_read(b: bytes, i: int):
    tag = b[i]
    ln = b[i + 1]
    i += 2
    if ln & 0x80:
        nb = ln & 0x7F
        ln = int.from_bytes(b[i: i + nb], "big")
        i += nb
    return tag, b[i: i + ln], i + ln


def rsa_from_pem(pem: str):
    """SubjectPublicKeyInfo or PKCS#1 RSAPublicKey PEM -> (n, e)."""
    body = "".join(l for l in pem.strip().splitlines() if not l.startswith("-----"))
    der = base64.b64decode(body)
    tag, seq, _ = _der_read(der, 0)
    tag1, first, nxt = _der_read(seq, 0)
    if tag1 == 0x30:  # SPKI: AlgorithmIdentifier, BIT STRING(RSAPublicKey)
        _, bits, _ = _der_read(seq, nxt)
        _, rsa, _ = _der_read(bits[1:], 0)
        _, nb, j = _der_read(rsa, 0)
        _, eb, _ = _der_read(rsa, j)
    else:
        nb = first
        _, eb, _ = _der_read(seq, nxt)
    return int.from_bytes(nb, "big"), int.from_bytes(eb, "big")


def rsa_from_jwk(jwk: dict):
    return int.from_bytes(_b64url(jwk["n"]), "big"), int.from_bytes(_b64url(jwk["e"]), "big")


# ---------------------------------------------------------------- JWT
class JwtError(Exception):
    pass


_ALLOWED_ALGS = ("HS256", "HS384", "HS512", "RS256", "RS384", "RS512")


def decode_jwt(token: str, *, secret: Optional[bytes] = None, rsa_key=None,
               jwks_fetch: Optional[Callable[[dict], Optional[tuple]]] = None, leeway: int = 0) -> dict:
    try:
        h64, p64, s64 = token.split(".")
        header = json.loads(_b64url(h64))
        payload = json.loads(_b64url(p64))
        sig = _b64url(s64)
    except Exception as e:  # noqa: BLE001
        raise JwtError(f"malformed token: {e}") from e
    alg = header.get("alg", "")
    if alg not in _ALLOWED_ALGS:
        raise JwtError(f"unsupported alg {alg!r}")
    signing_input = f"{h64}.{p64}".encode()
    if alg.startswith("HS"):
        if secret is None:
            raise JwtError("HMAC token but no secret-key configured")
        mac = hmac.new(secret, signing_input, getattr(hashlib, "sha" + alg[2:])).digest()
        if not hmac.compare_digest(mac, sig):
            raise JwtError("bad signature")
    else:
        key = rsa_key
        if key is None and jwks_fetch is not None:
            key = jwks_fetch(header)
        if key is None:
            raise JwtError("RSA token but no public key available")
        if not rsa_pkcs1_verify(key[0], key[1], signing_input, sig, "SHA" + alg[2:]):
            raise JwtError("bad signature")
    now = time.time()
    if "exp" in payload and now > float(payload["exp"]) + leeway:
        raise JwtError("token expired")
    if "nbf" in payload and now + leeway < float(payload["nbf"]):
        raise JwtError("token not yet valid")
    return payload


def encode_jwt_hs256(payload: dict, secret: bytes) -> str:
    """Helper for tests and the CLI (`gateway` commands with a shared secret)."""
    enc = lambda b: base64.urlsafe_b64encode(b).rstrip(b"=").decode()  # noqa: E731
    h = enc(json.dumps({"alg": "HS256", "typ": "JWT"}).encode())
    p = enc(json.dumps(payload).encode())
    sig = hmac.new(secret, f"{h}.{p}".encode(), hashlib.sha256).digest()
    return f"{h}.{p}.{enc(sig)}"


# ---------------------------------------------------------------- JWKS cache
class _JwksCache:
    """Process-wide JWKS documents keyed by the (trusted) URI, with a TTL.

    Only configured URIs or allowlisted ``jku`` URIs reach it, so it cannot be grown by
    arbitrary tokens; a lock makes concurrent first fetches of one URI fetch once."""

    def __init__(self, ttl_s: float = 300.0, size: int = 64):
        self.ttl_s = ttl_s
        self.size = size
        self._lock = threading.Lock()
        self._docs: "OrderedDict[str, tuple]" = OrderedDict()

    def get(self, uri: str) -> dict:
        now = time.monotonic()
        with self._lock:
            hit = self._docs.get(uri)
            if hit is not None and now - hit[0] < self.ttl_s:
                return hit[1]
            import requests
            doc = requests.get(uri, timeout=10).json()
            self._docs[uri] = (now, doc)
            self._docs.move_to_end(uri)
            while len(self._docs) > self.size:
                self._docs.popitem(last=False)
            return doc

    def clear(self) -> None:
        with self._lock:
            self._docs.clear()


_JWKS_CACHE = _JwksCache()


# ---------------------------------------------------------------- providers
class AuthProvider:
    def __init__(self, configuration: Dict[str, Any]):
        self.cfg = dict(configuration or {})

    def authenticate(self, ctx) -> AuthResult:
        raise NotImplementedError


class HttpAuthProvider(AuthProvider):
    def authenticate(self, ctx) -> AuthResult:
        import requests
        path = str(_cfg(self.cfg, "path-template", "pathTemplate", default="")).replace("{tenant}", ctx.tenant)
        url = str(_cfg(self.cfg, "base-url", "baseUrl", default="")) + path
        headers = dict(_cfg(self.cfg, "headers", default={}) or {})
        headers["Authorization"] = "Bearer " + (ctx.credentials or "")
        accepted = [int(x) for x in _cfg(self.cfg, "accepted-statuses", "acceptedStatuses", default=[200, 201])]
        try:
            r = requests.get(url, headers=headers, timeout=30)
        except Exception as e:  # noqa: BLE001
            return AuthResult(False, str(e))
        if r.status_code in accepted:
            return AuthResult(True)
        return AuthResult(False, f"Http authentication failed: {r.status_code}")


class JwtAuthProvider(AuthProvider):
    def __init__(self, configuration):
        super().__init__(configuration)
        sk = _cfg(self.cfg, "secret-key", "secretKey")
        self.secret = None
        if sk:
            s = str(sk)
            self.secret = base64.b64decode(s[len("base64:"):]) if s.startswith("base64:") else s.encode()
        pk = _cfg(self.cfg, "public-key", "publicKey")
        self.rsa = rsa_from_pem(str(pk)) if pk else None
        self.jwks_uri = _cfg(self.cfg, "jwks-uri", "jwksUri")
        allow = str(_cfg(self.cfg, "jwks-hosts-allowlist", "jwksHostsAllowlist", default="") or "").strip()
        # a regex full-matched against the jku's parsed HOST only, like the reference's
        # Pattern.compile(hostsAllowlist).matcher(host).matches()
        # (JwksUriSigningKeyResolver.java:72-75,132); a comma list of such patterns is
        # accepted too.  Never a prefix test on the URL string: "https://issuer.example"
        # must not admit https://issuer.example.evil.com/ or https://issuer.example@evil.com/.
        self.jwks_hosts = []
        if allow:
            for pat in [allow] + [h.strip() for h in allow.split(",") if h.strip() and "," in allow]:
                try:
                    self.jwks_hosts.append(re.compile(pat))
                except re.error as e:
                    raise ValueError(f"invalid jwks-hosts-allowlist pattern {pat!r}: {e}") from e
        self.auth_claim = _cfg(self.cfg, "auth-claim", "authClaim", default="sub")
        self.audience = _cfg(self.cfg, "audience")
        self.audience_claim = _cfg(self.cfg, "audience-claim", "audienceClaim", default="aud")

    def _trusted_uri(self, header: dict) -> Optional[str]:
        """The JWKS URI to use for this token.

        A token-supplied ``jku`` is followed only when a non-empty allowlist matches its
        host (``JwksUriSigningKeyResolver.java:131-134`` throws 'Untrusted hostname' when
        the allowlist is missing); otherwise the configured ``jwks-uri`` is used."""
        jku = header.get("jku")
        if jku and jku != self.jwks_uri:
            try:
                host = urllib.parse.urlparse(str(jku)).hostname or ""
            except ValueError:
                host = ""
            if not host or not self.jwks_hosts or not any(p.fullmatch(host) for p in self.jwks_hosts):
                raise JwtError(f"Untrusted hostname {host!r} for jku")
            return str(jku)
        return self.jwks_uri

    def _jwks(self, header: dict) -> Optional[tuple]:
        uri = self._trusted_uri(header)
        if not uri:
            return None
        try:
            keys = _JWKS_CACHE.get(uri)
        except Exception as e:  # noqa: BLE001
            raise JwtError(f"cannot fetch JWKS from {uri}: {e}") from e
        for k in keys.get("keys", []):
            if header.get("kid") in (None, k.get("kid")) and k.get("kty") == "RSA":
                return rsa_from_jwk(k)
        return None

    def authenticate(self, ctx) -> AuthResult:
        try:
            claims = decode_jwt(ctx.credentials or "", secret=self.secret, rsa_key=self.rsa, jwks_fetch=self._jwks)
        except JwtError as e:
            return AuthResult(False, str(e))
        if self.audience is not None:
            aud = claims.get(self.audience_claim)
            auds = aud if isinstance(aud, list) else [aud]
            if self.audience not in auds:
                return AuthResult(False, "audience mismatch")
        values = {k: str(v) for k, v in claims.items() if isinstance(v, (str, int, float, bool))}
        if self.auth_claim in claims:
            values["subject"] = str(claims[self.auth_claim])
        return AuthResult(True, None, values)


class GitHubAuthProvider(AuthProvider):
    def authenticate(self, ctx) -> AuthResult:
        import requests
        try:
            r = requests.get("https://api.github.com/user", timeout=30,
                             headers={"Authorization": f"Bearer {ctx.credentials}",
                                      "Accept": "application/vnd.github+json"})
        except Exception as e:  # noqa: BLE001
            return AuthResult(False, str(e))
        if r.status_code != 200:
            return AuthResult(False, f"GitHub authentication failed: {r.status_code}")
        u = r.json()
        return AuthResult(True, None, {k: str(u.get(k)) for k in ("login", "id", "name", "email") if u.get(k)})


class GoogleAuthProvider(JwtAuthProvider):
    GOOGLE_JWKS = "https://www.googleapis.com/oauth2/v3/certs"

    def __init__(self, configuration):
        super().__init__(configuration)
        self.jwks_uri = self.jwks_uri or self.GOOGLE_JWKS
        self.jwks_hosts = []  # Google's provider never trusts token-supplied key URIs
        self.audience = _cfg(self.cfg, "clientId", "client-id")

    def authenticate(self, ctx) -> AuthResult:
        res = super().authenticate(ctx)
        if res.authenticated:
            pv = res.principal_values
            res.principal_values = {k: pv[k] for k in ("subject", "email", "name", "locale") if k in pv}
        return res


PROVIDERS: Dict[str, Callable[[Dict[str, Any]], AuthProvider]] = {
    "http": HttpAuthProvider, "jwt": JwtAuthProvider, "github": GitHubAuthProvider, "google": GoogleAuthProvider,
}


def load_provider(name: str, configuration: Dict[str, Any]) -> AuthProvider:
    f = PROVIDERS.get(name)
    if f is None:
        raise ValueError(f"unknown gateway authentication provider {name}; known: {sorted(PROVIDERS)}")
    return f(configuration)


class _ProviderCache:
    """One provider instance per (provider, configuration): the gateway authenticates
    every request, and building a provider per request would drop its state."""

    def __init__(self, size: int = 256):
        self._lock = threading.Lock()
        self._items: "OrderedDict[str, AuthProvider]" = OrderedDict()
        self._size = size

    def get(self, name: str, configuration: Dict[str, Any]) -> AuthProvider:
        key = name + "\x00" + json.dumps(configuration or {}, sort_keys=True, default=str)
        with self._lock:
            p = self._items.get(key)
            if p is not None:
                self._items.move_to_end(key)
                return p
        p = load_provider(name, configuration)
        with self._lock:
            self._items[key] = p
            while len(self._items) > self._size:
                self._items.popitem(last=False)
        return p


PROVIDER_CACHE = _ProviderCache()
