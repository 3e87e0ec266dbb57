"""Control-plane authentication and authorization.

Reference behaviour, re-implemented (no JVM, no crypto library offline):

* ``langstream-auth-jwt/.../AuthenticationProviderToken.java:71-238`` -- a bearer token is
  a JWS verified with, in this order of preference:
  1. the keys at the token's ``jwks_uri`` CLAIM, only when the URL's host full-matches
     the ``jwks-hosts-allowlist`` regex (``JwksUriSigningKeyResolver.java:95-150``: no
     allowlist -> 'Untrusted hostname');
  2. the local Kubernetes API's keys when the token's ``iss`` equals the cluster's own
     issuer (``LocalKubernetesJwksUriSigningKeyResolver.java``: the issuer and its
     ``jwks_uri`` come from ``/.well-known/openid-configuration``, fetched with the pod's
     service-account token and verified against the pod's service-account CA bundle);
     no host check for that URI;
  3. the configured ``secret-key`` (HMAC) or ``public-key`` (X.509 SubjectPublicKeyInfo,
     RSA or EC by ``public-alg``, default RS256).
  Keys are read like ``readKeyFromUrl``: ``data:`` / ``file:`` URLs, a path to an
  existing file, or a base64 string.  JWKS keys must carry ``alg == public-alg``; the
  header's ``kid`` picks one.
* audience: when ``audience-claim`` is set, ``audience`` is required; the claim must be
  present and equal (string) or contain (list) the audience.
* principal (the "role"): the ``kubernetes.io.namespace`` claim minus
  ``kubernetes-namespace-prefix`` when ``allow-kubernetes-service-accounts`` is on, else the
  ``auth-claim`` (default ``sub``; a list claim gives its first string).
* ``TokenAuthFilter.java:84-97``: a principal listed in ``admin-roles`` gets ROLE_ADMIN.
* ``SecurityConfiguration.java:67-92``: ``/api/tenants/**`` needs ROLE_ADMIN, every other
  ``/api/**`` and ``/management/**`` route an authenticated principal, except the
  health / info / prometheus probes and the API docs.
* ``ApplicationResource.java:94-125`` / ``ArchetypeResource.java:59-90``
  (``performAuthorization``): an application, log, code or archetype call on tenant T is
  allowed for ROLE_ADMIN or for principal == T, else 403.

Signature algorithms: HS256/384/512, RS256/384/512 (PKCS#1 v1.5) and ES256/384/512
(ECDSA over P-256/P-384/P-521, raw r||s as JWS specifies), verified in pure Python.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import os
import re
import threading
import time
import urllib.parse
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..gateway.auth import _b64url, _der_read, rsa_pkcs1_verify

ROLE_ADMIN = "ROLE_ADMIN"
DEFAULT_K8S_TOKEN_PATH = "/var/run/secrets/kubernetes.io/serviceaccount/token"
DEFAULT_K8S_CA_PATH = "/var/run/secrets/kubernetes.io/serviceaccount/ca.crt"
DEFAULT_K8S_BASE_URL = "https://kubernetes.default.svc.cluster.local"


class AuthenticationError(Exception):
    """Token missing, malformed, unverifiable, expired, wrong audience or no principal."""


# ---------------------------------------------------------------- ECDSA (NIST prime curves)
@dataclass(frozen=True)
class _Curve:
    name: str
    p: int
    a: int
    b: int
    n: int
    gx: int
    gy: int
    size: int          # coordinate / scalar bytes
    hash: str


_P256 = _Curve("P-256", 0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF,
               -3, 0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B,
               0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551,
               0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
               0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5, 32, "sha256")
_P384 = _Curve("P-384", int("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFE"
                            "FFFFFFFF0000000000000000FFFFFFFF", 16), -3,
               int("B3312FA7E23EE7E4988E056BE3F82D19181D9C6EFE8141120314088F5013875A"
                   "C656398D8A2ED19D2A85C8EDD3EC2AEF", 16),
               int("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFC7634D81F4372DDF"
                   "581A0DB248B0A77AECEC196ACCC52973", 16),
               int("AA87CA22BE8B05378EB1C71EF320AD746E1D3B628BA79B9859F741E082542A38"
                   "5502F25DBF55296C3A545E3872760AB7", 16),
               int("3617DE4A96262C6F5D9E98BF9292DC29F8F41DBD289A147CE9DA3113B5F0B8C0"
                   "0A60B1CE1D7E819D7A431D7C90EA0E5F", 16), 48, "sha384")
_P521 = _Curve("P-521", (1 << 521) - 1, -3,
               int("0051953EB9618E1C9A1F929A21A0B68540EEA2DA725B99B315F3B8B489918EF1"
                   "09E156193951EC7E937B1652C0BD3BB1BF073573DF883D2C34F1EF451FD46B503F00", 16),
               int("01FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFA"
                   "51868783BF2F966B7FCC0148F709A5D03BB5C9B8899C47AEBB6FB71E91386409", 16),
               int("00C6858E06B70404E9CD9E3ECB662395B4429C648139053FB521F828AF606B4D3D"
                   "BAA14B5E77EFE75928FE1DC127A2FFA8DE3348B3C1856A429BF97E7E31C2E5BD66", 16),
               int("011839296A789A3BC0045C8A5FB42C7D1BD998F54449579B446817AFBD17273E66"
                   "2C97EE72995EF42640C550B9013FAD0761353C7086A272C24088BE94769FD16650", 16),
               66, "sha512")
_CURVES = {"P-256": _P256, "P-384": _P384, "P-521": _P521}
_CURVE_OIDS = {bytes.fromhex("2a8648ce3d030107"): _P256, bytes.fromhex("2b81040022"): _P384,
               bytes.fromhex("2b81040023"): _P521}
_ALG_CURVE = {"ES256": _P256, "ES384": _P384, "ES512": _P521}
_SUPPORTED_ALGS = ("HS256", "HS384", "HS512", "RS256", "RS384", "RS512", "ES256", "ES384", "ES512")


def _ec_add(c: _Curve, P, Q):
    # Jacobian coordinates (X, Y, Z); None is the point at infinity
    if P is None:
        return Q
    if Q is None:
        return P
    p = c.p
    X1, Y1, Z1 = P
    X2, Y2, Z2 = Q
    Z1s, Z2s = Z1 * Z1 % p, Z2 * Z2 % p
    U1, U2 = X1 * Z2s % p, X2 * Z1s % p
    S1, S2 = Y1 * Z2s * Z2 % p, Y2 * Z1s * Z1 % p
    if U1 == U2:
        if S1 != S2:
            return None
        return _ec_double(c, P)
    H, R = (U2 - U1) % p, (S2 - S1) % p
    H2 = H * H % p
    H3 = H2 * H % p
    X3 = (R * R - H3 - 2 * U1 * H2) % p
    Y3 = (R * (U1 * H2 - X3) - S1 * H3) % p
    return (X3, Y3, H * Z1 * Z2 % p)


def _ec_double(c: _Curve, P):
    if P is None:
        return None
    p = c.p
    X, Y, Z = P
    if Y == 0:
        return None
    YY = Y * Y % p
    S = 4 * X * YY % p
    ZZ = Z * Z % p
    M = (3 * X * X + c.a * ZZ * ZZ) % p
    X3 = (M * M - 2 * S) % p
    Y3 = (M * (S - X3) - 8 * YY * YY) % p
    return (X3, Y3, 2 * Y * Z % p)


def _ec_affine(c: _Curve, P):
    if P is None:
        return None
    X, Y, Z = P
    zi = pow(Z, -1, c.p)
    zi2 = zi * zi % c.p
    return (X * zi2 % c.p, Y * zi2 * zi % c.p)


def ec_mul(c: _Curve, k: int, P: Tuple[int, int]):
    """k * P for an affine P; returns affine (x, y) or None."""
    R, Q = None, (P[0], P[1], 1)
    while k:
        if k & 1:
            R = _ec_add(c, R, Q)
        Q = _ec_double(c, Q)
        k >>= 1
    return _ec_affine(c, R)


def _on_curve(c: _Curve, x: int, y: int) -> bool:
    return 0 <= x < c.p and 0 <= y < c.p and (y * y - (x * x * x + c.a * x + c.b)) % c.p == 0


def _ec_hash_int(c: _Curve, msg: bytes) -> int:
    digest = hashlib.new(c.hash, msg).digest()
    z = int.from_bytes(digest, "big")
    excess = len(digest) * 8 - c.n.bit_length()
    return z >> excess if excess > 0 else z


def ecdsa_verify(c: _Curve, pub: Tuple[int, int], msg: bytes, sig: bytes) -> bool:
    if len(sig) != 2 * c.size or not _on_curve(c, *pub):
        return False
    r, s = int.from_bytes(sig[:c.size], "big"), int.from_bytes(sig[c.size:], "big")
    if not (1 <= r < c.n and 1 <= s < c.n):
        return False
    w = pow(s, -1, c.n)
    z = _ec_hash_int(c, msg)
    u1, u2 = z * w % c.n, r * w % c.n
    G = (c.gx, c.gy, 1)
    Q = (pub[0], pub[1], 1)
    # Shamir's trick: u1 G + u2 Q in one double-and-add walk
    R, GQ = None, _ec_add(c, G, Q)
    for i in range(max(u1.bit_length(), u2.bit_length()) - 1, -1, -1):
        R = _ec_double(c, R)
        b1, b2 = (u1 >> i) & 1, (u2 >> i) & 1
        if b1 and b2:
            R = _ec_add(c, R, GQ)
        elif b1:
            R = _ec_add(c, R, G)
        elif b2:
            R = _ec_add(c, R, Q)
    A = _ec_affine(c, R)
    return A is not None and A[0] % c.n == r


# ---------------------------------------------------------------- keys
@dataclass
class VerifyKey:
    kind: str                       # "hmac" | "rsa" | "ec"
    hmac_key: bytes = b""
    rsa: Optional[Tuple[int, int]] = None
    ec: Optional[Tuple[_Curve, Tuple[int, int]]] = None

    def verify(self, alg: str, signing_input: bytes, sig: bytes) -> bool:
        if alg.startswith("HS"):
            if self.kind != "hmac":
                return False
            mac = hmac.new(self.hmac_key, signing_input, getattr(hashlib, "sha" + alg[2:])).digest()
            return hmac.compare_digest(mac, sig)
        if alg.startswith("RS"):
            return self.kind == "rsa" and rsa_pkcs1_verify(self.rsa[0], self.rsa[1], signing_input, sig,
                                                           "SHA" + alg[2:])
        if alg.startswith("ES"):
            if self.kind != "ec" or _ALG_CURVE.get(alg) is not self.ec[0]:
                return False
            return ecdsa_verify(self.ec[0], self.ec[1], signing_input, sig)
        return False


def read_key_bytes(conf: str) -> bytes:
    """``AuthenticationProviderToken.readKeyFromUrl``: data: / file: URL, an existing
    file, or base64 text."""
    if conf.startswith("data:"):
        meta, _, data = conf[5:].partition(",")
        if meta.endswith(";base64"):
            return base64.b64decode(data)
        return urllib.parse.unquote_to_bytes(data)
    if conf.startswith("file:"):
        with open(urllib.parse.urlparse(conf).path, "rb") as f:
            return f.read()
    if os.path.isfile(conf):
        with open(conf, "rb") as f:
            return f.read()
    if re.fullmatch(r"[A-Za-z0-9+/=\s]+", conf):
        try:
            return base64.b64decode(conf + "=" * (-len(conf.strip()) % 4))
        except Exception as e:  # noqa: BLE001
            raise ValueError(f"Illegal base64 character or key file {conf} doesn't exist") from e
    raise ValueError(f"Secret/Public key file {conf} doesn't exist")


def _pem_or_der(data: bytes) -> bytes:
    text = data.strip()
    if text.startswith(b"-----"):
        return base64.b64decode(b"".join(l for l in text.splitlines() if not l.startswith(b"-----")))
    return data


def public_key_from_spki(data: bytes, alg: str) -> VerifyKey:
    """X.509 SubjectPublicKeyInfo (DER or PEM) -> an RSA or EC verification key; the
    family must match ``alg`` like ``keyTypeForSignatureAlgorithm``."""
    der = _pem_or_der(data)
    _, spki, _ = _der_read(der, 0)
    _, algid, nxt = _der_read(spki, 0)
    _, bits, _ = _der_read(spki, nxt)
    _, oid, j = _der_read(algid, 0)
    if oid == bytes.fromhex("2a864886f70d010101"):             # rsaEncryption
        if not alg.startswith("RS"):
            raise ValueError(f"public key is RSA but public-alg is {alg}")
        _, rsa, _ = _der_read(bits[1:], 0)
        _, nb, k = _der_read(rsa, 0)
        _, eb, _ = _der_read(rsa, k)
        return VerifyKey("rsa", rsa=(int.from_bytes(nb, "big"), int.from_bytes(eb, "big")))
    if oid == bytes.fromhex("2a8648ce3d0201"):                 # id-ecPublicKey
        _, curve_oid, _ = _der_read(algid, j)
        c = _CURVE_OIDS.get(curve_oid)
        if c is None or _ALG_CURVE.get(alg) is not c:
            raise ValueError(f"EC public key curve does not match public-alg {alg}")
        pt = bits[1:]
        if pt[:1] != b"\x04" or len(pt) != 1 + 2 * c.size:
            raise ValueError("EC public key: uncompressed point expected")
        return VerifyKey("ec", ec=(c, (int.from_bytes(pt[1:1 + c.size], "big"),
                                       int.from_bytes(pt[1 + c.size:], "big"))))
    raise ValueError(f"The {alg} algorithm does not support this key type")


def key_from_jwk(jwk: Dict[str, Any]) -> Optional[VerifyKey]:
    kty = jwk.get("kty")
    if kty == "RSA":
        return VerifyKey("rsa", rsa=(int.from_bytes(_b64url(jwk["n"]), "big"),
                                     int.from_bytes(_b64url(jwk["e"]), "big")))
    if kty == "EC" and jwk.get("crv") in _CURVES:
        c = _CURVES[jwk["crv"]]
        return VerifyKey("ec", ec=(c, (int.from_bytes(_b64url(jwk["x"]), "big"),
                                       int.from_bytes(_b64url(jwk["y"]), "big"))))
    return None


# ---------------------------------------------------------------- the token authenticator
@dataclass
class TokenProperties:
    """``application.security.token.*`` (``AuthTokenProperties.java``)."""
    secret_key: Optional[str] = None
    public_key: Optional[str] = None
    auth_claim: Optional[str] = None
    public_alg: Optional[str] = None
    audience_claim: Optional[str] = None
    audience: Optional[str] = None
    admin_roles: List[str] = field(default_factory=list)
    jwks_hosts_allowlist: Optional[str] = None
    allow_kubernetes_service_accounts: bool = False
    kubernetes_namespace_prefix: str = "langstream-"
    # where the local Kubernetes API, the pod's service-account token and its CA bundle
    # are (tests point these at fakes); a None base URL disables the local-issuer path
    kubernetes_base_url: Optional[str] = DEFAULT_K8S_BASE_URL
    kubernetes_token_path: Optional[str] = DEFAULT_K8S_TOKEN_PATH
    kubernetes_ca_path: Optional[str] = DEFAULT_K8S_CA_PATH

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "TokenProperties":
        def g(*names, default=None):
            for n in names:
                if d.get(n) is not None:
                    return d[n]
            return default
        roles = g("admin-roles", "adminRoles", "admin_roles", default=[]) or []
        if isinstance(roles, str):
            roles = [r.strip() for r in roles.split(",") if r.strip()]
        allow_k8s = g("allow-kubernetes-service-accounts", "allowKubernetesServiceAccounts",
                      "allow_kubernetes_service_accounts", default=False)
        return cls(secret_key=g("secret-key", "secretKey", "secret_key"),
                   public_key=g("public-key", "publicKey", "public_key"),
                   auth_claim=g("auth-claim", "authClaim", "auth_claim"),
                   public_alg=g("public-alg", "publicAlg", "public_alg"),
                   audience_claim=g("audience-claim", "audienceClaim", "audience_claim"),
                   audience=g("audience"),
                   admin_roles=list(roles),
                   jwks_hosts_allowlist=g("jwks-hosts-allowlist", "jwksHostsAllowlist", "jwks_hosts_allowlist"),
                   allow_kubernetes_service_accounts=str(allow_k8s).lower() in ("1", "true", "yes"),
                   kubernetes_namespace_prefix=g("kubernetes-namespace-prefix", "kubernetesNamespacePrefix",
                                                 "kubernetes_namespace_prefix", default="langstream-"),
                   kubernetes_base_url=g("kubernetes-base-url", "kubernetes_base_url", default=DEFAULT_K8S_BASE_URL),
                   kubernetes_token_path=g("kubernetes-token-path", "kubernetes_token_path",
                                           default=DEFAULT_K8S_TOKEN_PATH),
                   kubernetes_ca_path=g("kubernetes-ca-path", "kubernetes_ca_path", default=DEFAULT_K8S_CA_PATH))


class TokenAuthenticator:
    """``AuthenticationProviderToken`` + the ROLE_ADMIN mapping of ``TokenAuthFilter``.

    ``http_get(url, headers) -> (status, parsed JSON or text)`` is injectable (tests)."""

    def __init__(self, props: TokenProperties, http_get: Optional[Callable[..., Tuple[int, Any]]] = None):
        self.p = props
        self.http_get = http_get or self._http_get_json
        self.public_alg = (props.public_alg or "RS256").strip()
        if self.public_alg not in _SUPPORTED_ALGS[3:]:
            raise ValueError(f"invalid algorithm provided {self.public_alg}")
        self.role_claim = props.auth_claim.strip() if props.auth_claim and props.auth_claim.strip() else "sub"
        self.audience_claim = props.audience_claim.strip() if props.audience_claim and props.audience_claim.strip() \
            else None
        self.audience = props.audience.strip() if props.audience and props.audience.strip() else None
        if self.audience_claim is not None and self.audience is None:
            raise ValueError(f"Token Audience Claim [{self.audience_claim}] configured, but Audience not")
        allow = (props.jwks_hosts_allowlist or "").strip()
        self.hosts_allowlist = re.compile(allow) if allow else None
        self.fallback: Optional[VerifyKey] = None
        if props.secret_key and str(props.secret_key).strip():
            self.fallback = VerifyKey("hmac", hmac_key=read_key_bytes(str(props.secret_key).strip()))
        elif props.public_key and str(props.public_key).strip():
            self.fallback = public_key_from_spki(read_key_bytes(str(props.public_key).strip()), self.public_alg)
        self.admin_roles = set(props.admin_roles or [])
        self._lock = threading.Lock()
        self._keys: Dict[Tuple[str, Optional[str]], VerifyKey] = {}
        self._k8s_token = self._read_file(props.kubernetes_token_path)
        self._k8s_issuer_loaded = False
        self._k8s_issuer: Optional[str] = None
        self._k8s_jwks: Dict[str, str] = {}

    @staticmethod
    def _read_file(path: Optional[str]) -> Optional[str]:
        if path and os.path.isfile(path):
            with open(path) as f:
                return f.read().strip()
        return None

    def _http_get_json(self, url: str, headers: Optional[Dict[str, str]] = None) -> Tuple[int, Any]:
        import requests
        # calls to the in-cluster API server are verified against the pod's service-account
        # CA bundle when one is mounted; everything else against the system trust store
        ca = self.p.kubernetes_ca_path
        base = self.p.kubernetes_base_url or ""
        verify: Any = True
        if ca and os.path.isfile(ca) and base and url.startswith(base):
            verify = ca
        r = requests.get(url, headers=headers or {}, timeout=30, verify=verify)
        try:
            body = r.json()
        except ValueError:
            body = r.text
        return r.status_code, body

    # -- the local Kubernetes issuer (LocalKubernetesJwksUriSigningKeyResolver)
    @staticmethod
    def _well_known(issuer: str) -> str:
        return issuer.rstrip("/") + "/.well-known/openid-configuration"

    def _auth_headers(self) -> Dict[str, str]:
        return {"Authorization": "Bearer " + self._k8s_token} if self._k8s_token else {}

    def _local_issuer(self) -> Optional[str]:
        with self._lock:
            if not self._k8s_issuer_loaded:
                self._k8s_issuer_loaded = True
                base = self.p.kubernetes_base_url
                if base:
                    try:
                        st, body = self.http_get(self._well_known(base), self._auth_headers())
                        if st == 200 and isinstance(body, dict) and body.get("issuer"):
                            self._k8s_issuer = str(body["issuer"])
                    except Exception:  # noqa: BLE001 - not in a pod: no local issuer
                        self._k8s_issuer = None
            return self._k8s_issuer

    def _jwks_uri_from_issuer(self, issuer: str) -> Optional[str]:
        local = self._local_issuer()
        if local is None or issuer != local:
            return None
        with self._lock:
            if issuer in self._k8s_jwks:
                return self._k8s_jwks[issuer]
        st, body = self.http_get(self._well_known(issuer), self._auth_headers())
        if st != 200 or not isinstance(body, dict) or not body.get("jwks_uri"):
            raise AuthenticationError(f"cannot read the jwks_uri of issuer {issuer}")
        with self._lock:
            self._k8s_jwks[issuer] = str(body["jwks_uri"])
        return str(body["jwks_uri"])

    # -- key resolution (JwksUriSigningKeyResolver.resolveSigningKey)
    def _fetch_jwks(self, uri: str, check_host: bool, with_token: bool) -> Dict[str, Any]:
        if check_host:
            try:
                host = urllib.parse.urlparse(uri).hostname or ""
            except ValueError:
                host = ""
            if self.hosts_allowlist is None or not self.hosts_allowlist.fullmatch(host):
                raise AuthenticationError(f"Untrusted hostname: '{host}'")
        st, body = self.http_get(uri, {})
        if st != 200 and with_token and self._k8s_token:
            st, body = self.http_get(uri, self._auth_headers())
        if st != 200 or not isinstance(body, dict):
            raise AuthenticationError(f"Failed to fetch keys from URL: {uri}, got {st}")
        return body

    def _jwks_key(self, uri: str, kid: Optional[str], check_host: bool, with_token: bool) -> VerifyKey:
        ck = (uri, kid)
        with self._lock:
            k = self._keys.get(ck)
        if k is not None:
            return k
        doc = self._fetch_jwks(uri, check_host, with_token)
        for jwk in doc.get("keys", []):
            if jwk.get("alg") != self.public_alg:
                continue
            if kid is not None and kid != jwk.get("kid"):
                continue
            k = key_from_jwk(jwk)
            if k is None:
                raise AuthenticationError(f"Failed to parse public key '{jwk.get('kid')}' from {uri}")
            with self._lock:
                self._keys[ck] = k
            return k
        raise AuthenticationError(f"No valid keys found from URL: {uri}, keyId: {kid}")

    def _resolve_key(self, header: Dict[str, Any], claims: Dict[str, Any]) -> Optional[VerifyKey]:
        uri = claims.get("jwks_uri")
        if isinstance(uri, str) and uri:
            return self._jwks_key(uri, header.get("kid"), True, False)
        iss = claims.get("iss")
        if isinstance(iss, str) and iss:
            k8s_uri = self._jwks_uri_from_issuer(iss)
            if k8s_uri:
                return self._jwks_key(k8s_uri, header.get("kid"), False, True)
        return self.fallback

    # -- public API
    def authenticate(self, token: str) -> str:
        """Returns the principal ("role"); raises AuthenticationError."""
        try:
            h64, p64, s64 = token.split(".")
            header = json.loads(_b64url(h64))
            claims = json.loads(_b64url(p64))
            sig = _b64url(s64)
        except Exception as e:  # noqa: BLE001
            raise AuthenticationError(f"Failed to authentication token: malformed ({e})") from e
        if not isinstance(header, dict) or not isinstance(claims, dict):
            raise AuthenticationError("Failed to authentication token: malformed")
        alg = header.get("alg", "")
        if alg not in _SUPPORTED_ALGS:
            raise AuthenticationError(f"Failed to authentication token: unsupported alg {alg!r}")
        key = self._resolve_key(header, claims)
        if key is None:
            raise AuthenticationError("Failed to authentication token: no signing key")
        if not key.verify(alg, f"{h64}.{p64}".encode(), sig):
            raise AuthenticationError("Failed to authentication token: bad signature")
        now = time.time()
        try:
            if "exp" in claims and now > float(claims["exp"]):
                raise AuthenticationError("Failed to authentication token: token expired")
            if "nbf" in claims and now < float(claims["nbf"]):
                raise AuthenticationError("Failed to authentication token: token not yet valid")
        except (TypeError, ValueError) as e:
            raise AuthenticationError(f"Failed to authentication token: bad exp/nbf ({e})") from e
        if self.audience_claim is not None:
            aud = claims.get(self.audience_claim)
            if aud is None:
                raise AuthenticationError(f"Found null Audience in token, for claimed field: {self.audience_claim}")
            if isinstance(aud, list):
                if not any(a == self.audience for a in aud):
                    raise AuthenticationError(f"Audiences in token: [{', '.join(map(str, aud))}] "
                                              f"not contains this broker: {self.audience}")
            elif not isinstance(aud, str):
                raise AuthenticationError(f"Audiences in token is not in expected format: {aud}")
            elif aud != self.audience:
                raise AuthenticationError(f"Audiences in token: [{aud}] not contains this broker: {self.audience}")
        principal = self._principal(claims)
        if principal is None:
            raise AuthenticationError("Token was valid, however no principal found.")
        return principal

    def _principal(self, claims: Dict[str, Any]) -> Optional[str]:
        if self.p.allow_kubernetes_service_accounts and isinstance(claims.get("kubernetes.io"), dict):
            ns = claims["kubernetes.io"].get("namespace")
            pref = self.p.kubernetes_namespace_prefix or ""
            if isinstance(ns, str) and ns.startswith(pref):
                return ns[len(pref):]
        v = claims.get(self.role_claim)
        if isinstance(v, str):
            return v
        if isinstance(v, list) and v and isinstance(v[0], str):
            return v[0]
        return None

    def is_admin(self, principal: str) -> bool:
        return principal in self.admin_roles


@dataclass
class Principal:
    name: str
    admin: bool


def authorize_tenant(principal: Optional[Principal], tenant: str) -> None:
    """``performAuthorization``: ROLE_ADMIN or principal == tenant (security off: None)."""
    if principal is None or principal.admin or principal.name == tenant:
        return
    raise PermissionError(f"principal {principal.name!r} is not allowed to access tenant {tenant!r}")


# routes open to anyone even with security on (SecurityConfiguration.java:70-91)
_PUBLIC = re.compile(r"^/(management/(health(/.*)?|info|prometheus)|api/docs|swagger-ui(/.*|\.html)?"
                     r"|v3/api-docs(/.*)?)$")


def route_policy(path: str, method: str) -> str:
    """'public' | 'admin' | 'authenticated' for a request path."""
    if method == "OPTIONS" or _PUBLIC.match(path):
        return "public"
    if path == "/api/tenants" or path.startswith("/api/tenants/"):
        return "admin"
    return "authenticated"
