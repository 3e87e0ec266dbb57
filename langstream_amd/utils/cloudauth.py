"""Cloud request signing without SDKs (none are installed offline):

* ``sigv4_headers`` -- AWS Signature Version 4 (header form) for any service; used by the
  S3 code storage / s3-source and the Bedrock provider (the reference uses the AWS SDK:
  BedrockServiceProvider.java, bedrock/BedrockClient.java:60-91).
* ``GoogleServiceAccount`` -- OAuth2 access tokens from a service-account JSON by the
  JWT-bearer grant (RS256-signed assertion -> ``token_uri``), refreshed ahead of expiry;
  the reference uses GoogleCredential.fromStream(...).createScoped(cloud-platform)
  (VertexAIProvider.java:108-140).  RSA signing is PKCS#1 v1.5 over SHA-256 with the key
  parsed from the PEM (PKCS#8 or PKCS#1 DER) -- pure Python big-int arithmetic.
"""
from __future__ import annotations

import base64
import datetime as _dt
import hashlib
import hmac
import json
import threading
import time
import urllib.parse
from typing import Dict, Optional, Tuple


# ---------------------------------------------------------------- AWS SigV4
def sigv4_headers(method: str, url: str, region: str, service: str, access_key: str, secret_key: str,
                  payload: bytes = b"", headers: Optional[Dict[str, str]] = None,
                  session_token: Optional[str] = None, now: Optional[_dt.datetime] = None) -> Dict[str, str]:
    """Headers (including ``Authorization``) that sign the request with SigV4."""
    u = urllib.parse.urlparse(url)
    now = now or _dt.datetime.now(_dt.timezone.utc)
    amz_date = now.strftime("%Y%m%dT%H%M%SZ")
    date = now.strftime("%Y%m%d")
    phash = hashlib.sha256(payload).hexdigest()
    hs = {k.lower(): str(v).strip() for k, v in (headers or {}).items()}
    hs["host"] = u.netloc
    hs["x-amz-date"] = amz_date
    if service == "s3":
        hs["x-amz-content-sha256"] = phash
    if session_token:
        hs["x-amz-security-token"] = session_token
    q = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
    canon_q = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}"
                       for k, v in sorted(q))
    signed = ";".join(sorted(hs))
    canon_h = "".join(f"{k}:{hs[k]}\n" for k in sorted(hs))
    path = u.path or "/"
    if service != "s3":   # every non-S3 service double-encodes the path
        path = urllib.parse.quote(path, safe="/-_.~%")
        path = urllib.parse.quote(path, safe="/-_.~")
    else:
        path = urllib.parse.quote(path, safe="/-_.~")
    canon = "\n".join([method.upper(), path, canon_q, canon_h, signed, phash])
    scope = f"{date}/{region}/{service}/aws4_request"
    sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canon.encode()).hexdigest()])

    def h(k, m):
        return hmac.new(k, m.encode(), hashlib.sha256).digest()

    key = h(h(h(h(("AWS4" + secret_key).encode(), date), region), service), "aws4_request")
    sig = hmac.new(key, sts.encode(), hashlib.sha256).hexdigest()
    out = {k: v for k, v in hs.items() if k != "host"}
    out["Authorization"] = f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, SignedHeaders={signed}, Signature={sig}"
    return out


# ---------------------------------------------------------------- RSA (PKCS#1 v1.5, SHA-256)
def _der_read(b: bytes, pos: int) -> Tuple[int, int, int]:
    """-> (tag, content start, content end)"""
    tag = b[pos]
    ln = b[pos + 1]
    pos += 2
    if ln & 0x80:
        n = ln & 0x7F
        ln = int.from_bytes(b[pos:pos + n], "big")
        pos += n
    return tag, pos, pos + ln


def _der_ints(b: bytes, pos: int, end: int):
    out = []
    while pos < end:
        tag, s, e = _der_read(b, pos)
        if tag == 0x02:
            out.append(int.from_bytes(b[s:e], "big"))
        pos = e
    return out


def rsa_private_key_from_pem(pem: str) -> Tuple[int, int]:
    """(n, d) from a PKCS#8 ``PRIVATE KEY`` or PKCS#1 ``RSA PRIVATE KEY`` PEM."""
    lines = [ln for ln in pem.strip().splitlines() if ln and not ln.startswith("-----")]
    der = base64.b64decode("".join(lines))
    tag, s, e = _der_read(der, 0)
    if "BEGIN RSA PRIVATE KEY" not in pem:          # PKCS#8: SEQ { version, algId, OCTET STRING { RSAPrivateKey } }
        pos = s
        _, _, pos = _der_read(der, pos)             # version
        _, _, pos = _der_read(der, pos)             # algorithm identifier
        tag, s2, e2 = _der_read(der, pos)
        if tag != 0x04:
            raise ValueError("unexpected PKCS#8 structure")
        der = der[s2:e2]
        tag, s, e = _der_read(der, 0)
    ints = _der_ints(der, s, e)                    # version, n, e, d, p, q, dp, dq, qinv
    return ints[1], ints[3]


_SHA256_PREFIX = bytes.fromhex("3031300d060960864801650304020105000420")


def rsa_sign_sha256(n: int, d: int, msg: bytes) -> bytes:
    k = (n.bit_length() + 7) // 8
    t = _SHA256_PREFIX + hashlib.sha256(msg).digest()
    em = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
    return pow(int.from_bytes(em, "big"), d, n).to_bytes(k, "big")


def _b64url(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


class GoogleServiceAccount:
    SCOPE = "https://www.googleapis.com/auth/cloud-platform"

    def __init__(self, service_account_json: str, scope: str = SCOPE):
        info = json.loads(service_account_json)
        self.email = info["client_email"]
        self.token_uri = info.get("token_uri", "https://oauth2.googleapis.com/token")
        self.n, self.d = rsa_private_key_from_pem(info["private_key"])
        self.key_id = info.get("private_key_id")
        self.scope = scope
        self._token: Optional[str] = None
        self._exp = 0.0
        self._lock = threading.Lock()

    def assertion(self, now: Optional[int] = None) -> str:
        now = int(now or time.time())
        header = {"alg": "RS256", "typ": "JWT"}
        if self.key_id:
            header["kid"] = self.key_id
        claims = {"iss": self.email, "scope": self.scope, "aud": self.token_uri, "iat": now, "exp": now + 3600}
        signing = _b64url(json.dumps(header).encode()) + "." + _b64url(json.dumps(claims).encode())
        return signing + "." + _b64url(rsa_sign_sha256(self.n, self.d, signing.encode()))

    def token(self) -> str:
        with self._lock:
            if self._token is None or time.time() > self._exp - 120:   # refresh 2 min ahead
                import requests
                r = requests.post(self.token_uri, data={"grant_type": "urn:ietf:params:oauth:grant-type:jwt-bearer",
                                                        "assertion": self.assertion()}, timeout=30)
                r.raise_for_status()
                j = r.json()
                self._token = j["access_token"]
                self._exp = time.time() + float(j.get("expires_in", 3600))
            return self._token
