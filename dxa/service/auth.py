"""Control-plane authentication and role checks (the reference's gateway + service host auth:
Services/DataX.Gateway/DataX.Gateway.Api/Controllers/GatewayController.cs:31-200, DataX.ServiceHost/.../
Authorization/DataXAuthConstants.cs:15-21, DataX.Utilities.Web/RolesCheck.cs — Reader/Writer app roles named
``DataXReader`` / ``DataXWriter``, a client whitelist of ``{objectId}.{tenantId}``, and a local-onebox bypass).

Modes (``DXA_AUTH``):
* ``jwt`` (the default whenever a key source is configured) — every request carries ``Authorization: Bearer <JWT>``;
  the token is verified here: RS256 against the JWKS of ``DXA_AUTH_JWKS`` (a file, an https URL, or
  ``aad:<tenant>`` for Azure AD's published keys) or HS256 with ``DXA_AUTH_HS256_SECRET``; ``exp`` / ``nbf`` (5 min
  skew), ``aud`` (``DXA_AUTH_AUDIENCE``) and ``iss`` (``DXA_AUTH_ISSUER``) are checked; the ``roles`` claim must hold
  the Reader role (read routes) or the Writer role (writes; Writer implies Reader), unless ``oid.tid`` is in
  ``DXA_AUTH_CLIENT_WHITELIST``.  With JWKS keys an audience is required (a tenant's signing keys also sign tokens
  issued for every other application in it; ``DXA_AUTH_ANY_AUDIENCE=1`` opts out), and only the configured role
  names count (RolesCheck.cs:20-21);
* ``local`` (the default with no key source: the onebox) — requests from the loopback interface pass, anything else
  gets 401 (RolesCheck.EnsureWriter(request, isLocal));
* ``gateway`` — behind a trusted gateway that already authenticated the caller: roles come from ``X-DXA-Roles``
  (the reference's UserRolesHeader) and requests without it are rejected;
* ``off`` — no checks (tests, development).
RSA verification is PKCS#1 v1.5 / SHA-256 with Python integers (no crypto package is available here).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import os
import threading
import time
from typing import Any, Dict, Iterable, Optional, Tuple

READER_ROLE = os.environ.get("DXA_READER_ROLE", "DataXReader")
WRITER_ROLE = os.environ.get("DXA_WRITER_ROLE", "DataXWriter")
SKEW_S = 300
_SHA256_DIGEST_INFO = bytes.fromhex("3031300d060960864801650304020105000420")


class AuthError(Exception):
    def __init__(self, status: int, msg: str):
        super().__init__(msg)
        self.status = status


def b64url_decode(s: str) -> bytes:
    s = s.strip()
    return base64.urlsafe_b64decode(s + "=" * (-len(s) % 4))


def b64url_encode(b: bytes) -> str:
    return base64.urlsafe_b64encode(b).rstrip(b"=").decode()


def _int(b64: str) -> int:
    return int.from_bytes(b64url_decode(b64), "big")


def rsa_verify_sha256(n: int, e: int, message: bytes, signature: bytes) -> bool:
    """PKCS#1 v1.5 RSASSA verification with SHA-256 (RFC 8017 §8.2.2)."""
    k = (n.bit_length() + 7) // 8
    if len(signature) != k:
        return False
    s = int.from_bytes(signature, "big")
    if s >= n:
        return False
    em = pow(s, e, n).to_bytes(k, "big")
    t = _SHA256_DIGEST_INFO + hashlib.sha256(message).digest()
    if k < len(t) + 11:
        return False
    expected = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
    return hmac.compare_digest(em, expected)


def rsa_sign_sha256(n: int, d: int, message: bytes) -> bytes:
    """The signing counterpart (tests and tooling that mint tokens for a local key)."""
    k = (n.bit_length() + 7) // 8
    t = _SHA256_DIGEST_INFO + hashlib.sha256(message).digest()
    em = b"\x00\x01" + b"\xff" * (k - len(t) - 3) + b"\x00" + t
    return pow(int.from_bytes(em, "big"), d, n).to_bytes(k, "big")


class KeySet:
    """RS256 public keys by ``kid`` from a JWKS document (file, URL, or ``aad:<tenant>``), refreshed hourly."""

    def __init__(self, source: str, ttl_s: float = 3600.0, min_refresh_s: float = 60.0):
        self.source = source
        self.ttl = ttl_s
        self.min_refresh = min_refresh_s      # an unknown ``kid`` re-reads the key set at most this often (a forged
        self._keys: Dict[Optional[str], Tuple[int, int]] = {}   # kid per request must not become a fetch per request)
        self._at = 0.0
        self._lock = threading.Lock()

    def _fetch(self) -> Dict[str, Any]:
        src = self.source
        if src.startswith("aad:"):
            src = f"https://login.microsoftonline.com/{src[4:]}/discovery/v2.0/keys"
        if src.startswith(("http://", "https://")):
            import urllib.request
            with urllib.request.urlopen(src, timeout=10) as r:
                return json.loads(r.read())
        with open(src) as f:
            return json.load(f)

    def get(self, kid: Optional[str]) -> Tuple[int, int]:
        with self._lock:
            age = time.time() - self._at
            if (not self._keys or age > self.ttl
                    or (kid is not None and kid not in self._keys and age > self.min_refresh)):
                doc = self._fetch()
                keys = {}
                for k in doc.get("keys", []):
                    if k.get("kty") == "RSA" and k.get("use", "sig") == "sig":
                        keys[k.get("kid")] = (_int(k["n"]), _int(k["e"]))
                self._keys, self._at = keys, time.time()
            if kid in self._keys:
                return self._keys[kid]
            if kid is None and len(self._keys) == 1:
                return next(iter(self._keys.values()))
        raise AuthError(401, f"unknown signing key {kid!r}")


def decode_jwt(token: str, keys: Optional[KeySet] = None, hs256_secret: Optional[bytes] = None,
               audience: Optional[str] = None, issuer: Optional[str] = None, now: Optional[float] = None
               ) -> Dict[str, Any]:
    """Verify a compact JWS and its time / audience / issuer claims → the claims."""
    try:
        h64, p64, s64 = token.split(".")
        header = json.loads(b64url_decode(h64))
        claims = json.loads(b64url_decode(p64))
        sig = b64url_decode(s64)
    except (ValueError, json.JSONDecodeError) as e:
        raise AuthError(401, f"malformed token: {e}")
    signed = f"{h64}.{p64}".encode()
    alg = header.get("alg")
    if alg == "RS256" and keys is not None:
        n, e = keys.get(header.get("kid"))
        if not rsa_verify_sha256(n, e, signed, sig):
            raise AuthError(401, "bad token signature")
    elif alg == "HS256" and hs256_secret is not None:
        if not hmac.compare_digest(hmac.new(hs256_secret, signed, hashlib.sha256).digest(), sig):
            raise AuthError(401, "bad token signature")
    else:
        raise AuthError(401, f"token algorithm {alg!r} not accepted")
    t = time.time() if now is None else now
    if "exp" in claims and t > float(claims["exp"]) + SKEW_S:
        raise AuthError(401, "token expired")
    if "nbf" in claims and t + SKEW_S < float(claims["nbf"]):
        raise AuthError(401, "token not yet valid")
    if audience is not None:
        aud = claims.get("aud")
        auds = aud if isinstance(aud, list) else [aud]
        if audience not in auds:
            raise AuthError(401, "token audience mismatch")
    if issuer is not None and claims.get("iss") != issuer:
        raise AuthError(401, "token issuer mismatch")
    return claims


class Authenticator:
    def __init__(self, env: Optional[Dict[str, str]] = None):
        env = dict(os.environ if env is None else env)
        jwks = env.get("DXA_AUTH_JWKS")
        secret = env.get("DXA_AUTH_HS256_SECRET")
        legacy = env.get("DXA_AUTH")
        mode = (legacy or "").lower()
        if mode == "1":                       # the round-2 switch: gateway roles header
            mode = "gateway"
        if not mode:
            mode = "jwt" if (jwks or secret) else "local"
        self.mode = mode
        self.keys = KeySet(jwks) if jwks else None
        self.secret = secret.encode() if secret else None
        self.audience = env.get("DXA_AUTH_AUDIENCE")
        self.issuer = env.get("DXA_AUTH_ISSUER")
        self.whitelist = {x.strip() for x in (env.get("DXA_AUTH_CLIENT_WHITELIST") or "").split(",") if x.strip()}
        if self.mode == "jwt" and not (self.keys or self.secret):
            raise ValueError("DXA_AUTH=jwt needs DXA_AUTH_JWKS or DXA_AUTH_HS256_SECRET")
        if self.mode == "jwt" and self.keys is not None and not self.audience \
                and env.get("DXA_AUTH_ANY_AUDIENCE") != "1":
            raise ValueError("DXA_AUTH_JWKS needs DXA_AUTH_AUDIENCE (the application's id URI): the key set also "
                             "signs tokens issued to other applications (DXA_AUTH_ANY_AUDIENCE=1 to accept any)")

    @staticmethod
    def _is_local(client_host: Optional[str]) -> bool:
        return client_host in ("127.0.0.1", "::1", "localhost")

    def check(self, need_writer: bool, authorization: Optional[str], roles_header: Optional[str],
              client_host: Optional[str]) -> Dict[str, Any]:
        """→ the caller's identity (claims); raises AuthError(401 / 403)."""
        if self.mode == "off":
            return {}
        if self.mode == "local":
            if self._is_local(client_host):
                return {}
            raise AuthError(401, "authentication is not configured: only local (onebox) requests are accepted")
        if self.mode == "gateway":
            if roles_header is None:
                raise AuthError(401, "missing roles header from the gateway")
            return self._roles_ok({"roles": [r.strip() for r in roles_header.split(",") if r.strip()]}, need_writer)
        if not authorization or not authorization.lower().startswith("bearer "):
            raise AuthError(401, "bearer token required")
        claims = decode_jwt(authorization[7:].strip(), self.keys, self.secret, self.audience, self.issuer)
        return self._roles_ok(claims, need_writer)

    def _roles_ok(self, claims: Dict[str, Any], need_writer: bool) -> Dict[str, Any]:
        roles = claims.get("roles") or []
        roles = [roles] if isinstance(roles, str) else list(roles)
        low = {r.lower() for r in roles}
        writer = WRITER_ROLE.lower() in low
        reader = writer or READER_ROLE.lower() in low
        who = f"{claims.get('oid', '')}.{claims.get('tid', '')}"
        if who in self.whitelist:
            return claims
        if need_writer and not writer:
            raise AuthError(403, f"{WRITER_ROLE} role needed to perform this action.  User has the following "
                                 f"roles: {','.join(roles)}")
        if not reader:
            raise AuthError(403, f"{READER_ROLE} role needed to perform this action")
        return claims


def make_token(claims: Dict[str, Any], alg: str = "HS256", secret: Optional[bytes] = None,
               rsa: Optional[Tuple[int, int]] = None, kid: Optional[str] = None) -> str:
    """Mint a JWT (tests / onebox tooling): HS256 with ``secret`` or RS256 with ``rsa=(n, d)``."""
    header = {"alg": alg, "typ": "JWT"}
    if kid:
        header["kid"] = kid
    h64 = b64url_encode(json.dumps(header, separators=(",", ":")).encode())
    p64 = b64url_encode(json.dumps(claims, separators=(",", ":")).encode())
    signed = f"{h64}.{p64}".encode()
    if alg == "HS256":
        sig = hmac.new(secret, signed, hashlib.sha256).digest()
    else:
        sig = rsa_sign_sha256(rsa[0], rsa[1], signed)
    return f"{h64}.{p64}.{b64url_encode(sig)}"
