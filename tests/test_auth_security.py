"""JWT provider hardening (gateway auth, G5/G6): token-supplied JWKS URIs are never
trusted without an allowlist, unknown algorithms are rejected as JwtError, providers
are cached per configuration."""
import base64
import json

import pytest

from langstream_amd.gateway import auth
from langstream_amd.gateway.auth import (PROVIDER_CACHE, JwtError, decode_jwt, encode_jwt_hs256, GoogleAuthProvider,
                                         JwtAuthProvider)


def _b64(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def _token(header: dict, payload: dict, sig: bytes = b"x" * 128) -> str:
    return ".".join([_b64(json.dumps(header).encode()), _b64(json.dumps(payload).encode()), _b64(sig)])


class _Ctx:
    def __init__(self, creds):
        self.credentials = creds
        self.tenant = "t"


@pytest.fixture
def fetched(monkeypatch):
    calls = []

    def fake_get(uri):
        calls.append(uri)
        return {"keys": []}

    monkeypatch.setattr(auth._JWKS_CACHE, "get", fake_get)
    return calls


def test_foreign_jku_without_allowlist_is_rejected(fetched):
    p = JwtAuthProvider({"jwks-uri": "https://issuer.example/jwks"})
    tok = _token({"alg": "RS256", "kid": "k1", "jku": "https://evil.example/jwks"}, {"sub": "admin"})
    res = p.authenticate(_Ctx(tok))
    assert not res.authenticated and "Untrusted" in res.reason
    assert fetched == []  # never fetched the attacker's URI


def test_foreign_jku_not_matching_allowlist_is_rejected(fetched):
    p = JwtAuthProvider({"jwks-uri": "https://issuer.example/jwks", "jwks-hosts-allowlist": "issuer.example"})
    tok = _token({"alg": "RS256", "jku": "https://evil.example/jwks"}, {"sub": "a"})
    assert not p.authenticate(_Ctx(tok)).authenticated
    assert fetched == []
    tok = _token({"alg": "RS256", "jku": "https://issuer.example/other"}, {"sub": "a"})
    p.authenticate(_Ctx(tok))
    assert fetched == ["https://issuer.example/other"]


def test_configured_uri_is_used_without_jku(fetched):
    p = JwtAuthProvider({"jwks-uri": "https://issuer.example/jwks"})
    res = p.authenticate(_Ctx(_token({"alg": "RS256"}, {"sub": "a"})))
    assert not res.authenticated
    assert fetched == ["https://issuer.example/jwks"]


def test_google_ignores_token_jku_even_with_allowlist(fetched):
    p = GoogleAuthProvider({"clientId": "c", "jwks-hosts-allowlist": "evil.example"})
    tok = _token({"alg": "RS256", "jku": "https://evil.example/jwks"}, {"aud": "c"})
    assert not p.authenticate(_Ctx(tok)).authenticated
    assert fetched == []


@pytest.mark.parametrize("alg", ["HS1", "HS", "HSxyz", "RS1", "none", "ES256", ""])
def test_unknown_alg_is_jwt_error(alg):
    with pytest.raises(JwtError):
        decode_jwt(_token({"alg": alg}, {"sub": "a"}), secret=b"k")


def test_hs256_roundtrip_and_provider_cache():
    tok = encode_jwt_hs256({"sub": "u1"}, b"secret")
    assert decode_jwt(tok, secret=b"secret")["sub"] == "u1"
    cfg = {"secret-key": "secret"}
    p1 = PROVIDER_CACHE.get("jwt", cfg)
    assert PROVIDER_CACHE.get("jwt", dict(cfg)) is p1
    assert PROVIDER_CACHE.get("jwt", {"secret-key": "other"}) is not p1
    res = p1.authenticate(_Ctx(tok))
    assert res.authenticated and res.principal_values["subject"] == "u1"


@pytest.mark.parametrize("jku", ["https://issuer.example.evil.com/jwks", "https://issuer.example@evil.com/jwks",
                                 "https://evil.com/issuer.example/jwks", "https://evil.com/?h=issuer.example"])
def test_jku_allowlist_is_a_host_fullmatch_not_a_prefix(fetched, jku):
    """the allowlist used to admit any jku whose URL string started with an
    entry; now it is a regex full-matched against the parsed host only."""
    for allow in ("https://issuer.example", "issuer.example", r"issuer\.example"):
        p = JwtAuthProvider({"jwks-uri": "https://issuer.example/jwks", "jwks-hosts-allowlist": allow})
        res = p.authenticate(_Ctx(_token({"alg": "RS256", "jku": jku}, {"sub": "a"})))
        assert not res.authenticated and "Untrusted" in res.reason, (allow, jku)
    assert fetched == []  # the attacker's JWKS is never fetched


def test_jku_allowlist_regex_matches_subdomains(fetched):
    p = JwtAuthProvider({"jwks-uri": "https://issuer.example.com/jwks", "jwks-hosts-allowlist": r".*\.example\.com"})
    assert p._trusted_uri({"jku": "https://keys.example.com/jwks"}) == "https://keys.example.com/jwks"
    with pytest.raises(JwtError):
        p._trusted_uri({"jku": "https://keys.example.com.evil.io/jwks"})
