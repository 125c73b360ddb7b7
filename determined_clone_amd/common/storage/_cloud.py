"""Object-store checkpoint backends spoken over their REST protocols (no vendor SDKs: boto3,
google-cloud-storage and azure-storage-blob are not part of the MI355X image).

Reference: ``harness/determined/common/storage/{s3,gcs,azure}.py`` (SDK based). Here:
* S3 (and S3-compatible endpoints: MinIO, Ceph RGW) -- AWS Signature Version 4 over ``requests``,
  ListObjectsV2 paging, per-object PUT / GET / DELETE;
* Azure Blob -- SharedKey (connection string ``AccountName`` / ``AccountKey``) or SAS token;
* GCS -- JSON API with an OAuth bearer token (``GOOGLE_OAUTH_ACCESS_TOKEN`` or the GCE metadata
  server); service-account key signing would need an RSA library the image does not ship.
All three share :class:`ObjectStorageManager` (checkpoint directory <-> key prefix mapping)."""
import base64
import datetime
import email.utils
import fnmatch
import hashlib
import hmac
import os
import pathlib
import time
import urllib.parse
import xml.etree.ElementTree as ET
from typing import Any, Dict, List, Optional, Tuple

import requests

from determined_clone_amd.common.storage import Selector, StorageManager

_CHUNK = 1 << 20


# ---------------------------------------------------------------------------- generic manager
class ObjectStore:
    """Minimal object-store protocol used by :class:`ObjectStorageManager`."""

    def put(self, key: str, path: str) -> None:
        raise NotImplementedError

    def get(self, key: str, path: str) -> None:
        raise NotImplementedError

    def list(self, prefix: str) -> List[Tuple[str, int]]:
        raise NotImplementedError

    def delete(self, key: str) -> None:
        raise NotImplementedError


class ObjectStorageManager(StorageManager):
    """Checkpoint ``storage_id`` = key prefix ``[<prefix>/]<storage_id>/`` in a bucket/container."""

    def __init__(self, store: ObjectStore, prefix: Optional[str] = None) -> None:
        super().__init__(prefix or "")
        self.store = store
        self.prefix = (prefix or "").strip("/")

    def _key(self, *parts: str) -> str:
        return "/".join(p.strip("/") for p in (self.prefix, *parts) if p and p.strip("/"))

    def upload(self, src: Any, dst: str, paths: Optional[List[str]] = None) -> None:
        src = pathlib.Path(src)
        rels = paths if paths is not None else [str(p.relative_to(src)) for p in src.rglob("*")]
        for rel in rels:
            p = src / rel
            if p.is_file():
                self.store.put(self._key(dst, rel), str(p))

    def _objects(self, storage_id: str) -> List[Tuple[str, int]]:
        base = self._key(storage_id) + "/"
        return [(k[len(base):], n) for k, n in self.store.list(base) if k.startswith(base)]

    def download(self, src: str, dst: Any, selector: Selector = None) -> None:
        objs = self._objects(src)
        if not objs:
            from determined_clone_amd.errors import CheckpointNotFoundException

            raise CheckpointNotFoundException(f"checkpoint {src} not found under {self._key(src)}/")
        for rel, _ in objs:
            if selector is not None and not selector(rel):
                continue
            d = pathlib.Path(dst) / rel
            d.parent.mkdir(parents=True, exist_ok=True)
            self.store.get(self._key(src, rel), str(d))

    def delete(self, storage_id: str, globs: Optional[List[str]] = None) -> Dict[str, int]:
        remaining: Dict[str, int] = {}
        for rel, n in self._objects(storage_id):
            if not globs or any(fnmatch.fnmatch(rel, g) or g == "**/*" for g in globs):
                self.store.delete(self._key(storage_id, rel))
            else:
                remaining[rel] = n
        return remaining

    def list_files(self, storage_id: str) -> Dict[str, int]:
        return dict(self._objects(storage_id))


def _sha256_file(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(_CHUNK), b""):
            h.update(chunk)
    return h.hexdigest()


def _stream_to(resp: requests.Response, path: str) -> None:
    with open(path, "wb") as f:
        for chunk in resp.iter_content(_CHUNK):
            f.write(chunk)


def _check(resp: requests.Response, what: str) -> requests.Response:
    if resp.status_code >= 300:
        raise RuntimeError(f"{what}: HTTP {resp.status_code}: {resp.text[:300]}")
    return resp


# ---------------------------------------------------------------------------- S3 / SigV4
EMPTY_SHA256 = hashlib.sha256(b"").hexdigest()


def _hmac(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode(), hashlib.sha256).digest()


def sigv4_headers(method: str, url: str, headers: Dict[str, str], payload_sha256: str,
                  access_key: str, secret_key: str, region: str, service: str,
                  amz_date: Optional[str] = None, session_token: Optional[str] = None) -> Dict[str, str]:
    """AWS Signature Version 4: returns ``headers`` plus ``x-amz-date`` and ``Authorization``.
    Every header passed in is signed (callers pass host and the x-amz-* headers)."""
    u = urllib.parse.urlsplit(url)
    amz_date = amz_date or datetime.datetime.now(datetime.timezone.utc).strftime("%Y%m%dT%H%M%SZ")
    out = dict(headers)
    out["x-amz-date"] = amz_date
    if session_token:
        out["x-amz-security-token"] = session_token
    out.setdefault("host", u.netloc)
    canon_h = {k.lower().strip(): " ".join(str(v).split()) for k, v in out.items()}
    signed = ";".join(sorted(canon_h))
    path = urllib.parse.quote(urllib.parse.unquote(u.path) or "/", safe="/~")
    query = urllib.parse.parse_qsl(u.query, keep_blank_values=True)
    canon_q = "&".join(f"{urllib.parse.quote(k, safe='~')}={urllib.parse.quote(v, safe='~')}"
                       for k, v in sorted(query))
    canon_req = "\n".join([method, path, canon_q,
                           "".join(f"{k}:{canon_h[k]}\n" for k in sorted(canon_h)), signed, payload_sha256])
    day = amz_date[:8]
    scope = f"{day}/{region}/{service}/aws4_request"
    to_sign = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canon_req.encode()).hexdigest()])
    k = _hmac(_hmac(_hmac(_hmac(("AWS4" + secret_key).encode(), day), region), service), "aws4_request")
    sig = hmac.new(k, to_sign.encode(), hashlib.sha256).hexdigest()
    out["Authorization"] = (f"AWS4-HMAC-SHA256 Credential={access_key}/{scope}, "
                            f"SignedHeaders={signed}, Signature={sig}")
    return out


def imds_credentials(http: requests.Session, imds: str = "http://169.254.169.254") -> Dict[str, Any]:
    """Instance-profile credentials from the EC2 metadata service (IMDSv2): the role the
    machine was launched with (``det deploy aws`` gives the master and agents one each).
    Returns ``{"access_key", "secret_key", "token", "expiry"}``."""
    imds = imds.rstrip("/")
    tok = http.put(f"{imds}/latest/api/token", timeout=5,
                   headers={"X-aws-ec2-metadata-token-ttl-seconds": "21600"}).text
    hdr = {"X-aws-ec2-metadata-token": tok}
    base = f"{imds}/latest/meta-data/iam/security-credentials/"
    role = http.get(base, headers=hdr, timeout=5).text.strip().splitlines()[0]
    c = http.get(base + role, headers=hdr, timeout=5).json()
    exp = time.time() + 3600.0
    if c.get("Expiration"):
        try:
            exp = datetime.datetime.fromisoformat(c["Expiration"].replace("Z", "+00:00")).timestamp()
        except ValueError:
            pass
    return {"access_key": c["AccessKeyId"], "secret_key": c["SecretAccessKey"], "token": c.get("Token"),
            "expiry": exp}


class S3Store(ObjectStore):
    def __init__(self, bucket: str, access_key: Optional[str] = None, secret_key: Optional[str] = None,
                 endpoint_url: Optional[str] = None, region: Optional[str] = None,
                 session: Optional[requests.Session] = None) -> None:
        self.bucket = bucket
        self.access_key = access_key or os.environ.get("AWS_ACCESS_KEY_ID", "")
        self.secret_key = secret_key or os.environ.get("AWS_SECRET_ACCESS_KEY", "")
        self.token = os.environ.get("AWS_SESSION_TOKEN")
        self.region = region or os.environ.get("AWS_REGION") or os.environ.get("AWS_DEFAULT_REGION") or "us-east-1"
        # path-style addressing works for AWS and every S3-compatible server
        self.endpoint = (endpoint_url or f"https://s3.{self.region}.amazonaws.com").rstrip("/")
        self.http = session or requests.Session()
        self.imds = os.environ.get("DET_AWS_IMDS_ENDPOINT", "http://169.254.169.254")
        self._expiry = 0.0  # > 0: credentials came from the instance profile and expire

    def _url(self, key: str = "", query: str = "") -> str:
        k = urllib.parse.quote(key, safe="/~")
        return f"{self.endpoint}/{self.bucket}" + (f"/{k}" if key else "") + (f"?{query}" if query else "")

    def _req(self, method: str, url: str, payload_sha: str = EMPTY_SHA256, **kw: Any) -> requests.Response:
        if (not self.access_key and not self._expiry) or (self._expiry and time.time() > self._expiry - 300):
            c = imds_credentials(self.http, self.imds)
            self.access_key, self.secret_key, self.token, self._expiry = (
                c["access_key"], c["secret_key"], c["token"], c["expiry"])
        h = sigv4_headers(method, url, {"x-amz-content-sha256": payload_sha}, payload_sha,
                          self.access_key, self.secret_key, self.region, "s3", session_token=self.token)
        return self.http.request(method, url, headers=h, **kw)

    def put(self, key: str, path: str) -> None:
        with open(path, "rb") as f:
            _check(self._req("PUT", self._url(key), _sha256_file(path), data=f), f"s3 put {key}")

    def get(self, key: str, path: str) -> None:
        _stream_to(_check(self._req("GET", self._url(key), stream=True), f"s3 get {key}"), path)

    def list(self, prefix: str) -> List[Tuple[str, int]]:
        out: List[Tuple[str, int]] = []
        token: Optional[str] = None
        while True:
            q = {"list-type": "2", "prefix": prefix}
            if token:
                q["continuation-token"] = token
            url = self._url(query=urllib.parse.urlencode(sorted(q.items()), quote_via=urllib.parse.quote))
            root = ET.fromstring(_check(self._req("GET", url), "s3 list").content)
            ns = root.tag[:root.tag.index("}") + 1] if root.tag.startswith("{") else ""
            for c in root.findall(f"{ns}Contents"):
                out.append((c.findtext(f"{ns}Key") or "", int(c.findtext(f"{ns}Size") or 0)))
            if (root.findtext(f"{ns}IsTruncated") or "false").lower() != "true":
                return out
            token = root.findtext(f"{ns}NextContinuationToken")

    def delete(self, key: str) -> None:
        _check(self._req("DELETE", self._url(key)), f"s3 delete {key}")


# ---------------------------------------------------------------------------- Azure Blob
def parse_connection_string(cs: str) -> Dict[str, str]:
    return dict(part.split("=", 1) for part in cs.split(";") if "=" in part)


def azure_shared_key(method: str, url: str, headers: Dict[str, str], account: str, key_b64: str) -> str:
    """``Authorization`` value for the Blob service SharedKey scheme."""
    u = urllib.parse.urlsplit(url)
    h = {k.lower(): str(v) for k, v in headers.items()}
    length = h.get("content-length", "")
    std = [method, h.get("content-encoding", ""), h.get("content-language", ""),
           "" if length == "0" else length, h.get("content-md5", ""), h.get("content-type", ""),
           h.get("date", ""), h.get("if-modified-since", ""), h.get("if-match", ""),
           h.get("if-none-match", ""), h.get("if-unmodified-since", ""), h.get("range", "")]
    canon_h = "".join(f"{k}:{h[k].strip()}\n" for k in sorted(k for k in h if k.startswith("x-ms-")))
    res = f"/{account}{urllib.parse.unquote(u.path) or '/'}"
    q: Dict[str, List[str]] = {}
    for k, v in urllib.parse.parse_qsl(u.query, keep_blank_values=True):
        q.setdefault(k.lower(), []).append(v)
    for k in sorted(q):
        res += f"\n{k}:{','.join(sorted(q[k]))}"
    to_sign = "\n".join(std) + "\n" + canon_h + res
    sig = base64.b64encode(hmac.new(base64.b64decode(key_b64), to_sign.encode(), hashlib.sha256).digest())
    return f"SharedKey {account}:{sig.decode()}"


class AzureBlobStore(ObjectStore):
    API_VERSION = "2021-08-06"

    def __init__(self, container: str, connection_string: Optional[str] = None,
                 account_url: Optional[str] = None, credential: Optional[str] = None,
                 session: Optional[requests.Session] = None) -> None:
        cs = parse_connection_string(connection_string or os.environ.get("AZURE_STORAGE_CONNECTION_STRING", ""))
        self.account = cs.get("AccountName", "")
        self.key = cs.get("AccountKey")
        self.sas = (cs.get("SharedAccessSignature") or (credential if credential and "sig=" in credential else "")).lstrip("?")
        if self.key is None and credential and "sig=" not in credential:
            self.key = credential
        endpoint = account_url or cs.get("BlobEndpoint")
        if not endpoint:
            suffix = cs.get("EndpointSuffix", "core.windows.net")
            endpoint = f"{cs.get('DefaultEndpointsProtocol', 'https')}://{self.account}.blob.{suffix}"
        self.endpoint = endpoint.rstrip("/")
        self.container = container
        self.http = session or requests.Session()

    def _url(self, blob: str = "", query: str = "") -> str:
        url = f"{self.endpoint}/{self.container}" + (f"/{urllib.parse.quote(blob, safe='/~')}" if blob else "")
        q = "&".join(x for x in (query, self.sas) if x)
        return url + (f"?{q}" if q else "")

    def _req(self, method: str, url: str, extra: Optional[Dict[str, str]] = None, **kw: Any) -> requests.Response:
        h = {"x-ms-date": email.utils.formatdate(usegmt=True), "x-ms-version": self.API_VERSION}
        h.update(extra or {})
        if self.key and not self.sas:
            h["Authorization"] = azure_shared_key(method, url, h, self.account, self.key)
        return self.http.request(method, url, headers=h, **kw)

    def put(self, key: str, path: str) -> None:
        size = os.path.getsize(path)
        with open(path, "rb") as f:
            _check(self._req("PUT", self._url(key), {"x-ms-blob-type": "BlockBlob", "Content-Length": str(size),
                                                      "Content-Type": "application/octet-stream"}, data=f),
                   f"azure put {key}")

    def get(self, key: str, path: str) -> None:
        _stream_to(_check(self._req("GET", self._url(key), stream=True), f"azure get {key}"), path)

    def list(self, prefix: str) -> List[Tuple[str, int]]:
        out: List[Tuple[str, int]] = []
        marker = ""
        while True:
            q = {"restype": "container", "comp": "list", "prefix": prefix}
            if marker:
                q["marker"] = marker
            root = ET.fromstring(_check(self._req("GET", self._url(query=urllib.parse.urlencode(q))), "azure list").content)
            for b in root.iter("Blob"):
                out.append((b.findtext("Name") or "", int(b.findtext("Properties/Content-Length") or 0)))
            marker = root.findtext("NextMarker") or ""
            if not marker:
                return out

    def delete(self, key: str) -> None:
        _check(self._req("DELETE", self._url(key)), f"azure delete {key}")


# ---------------------------------------------------------------------------- GCS (JSON API)
class GCSStore(ObjectStore):
    def __init__(self, bucket: str, endpoint_url: Optional[str] = None, token: Optional[str] = None,
                 session: Optional[requests.Session] = None) -> None:
        self.bucket = bucket
        self.endpoint = (endpoint_url or os.environ.get("STORAGE_EMULATOR_HOST") or "https://storage.googleapis.com").rstrip("/")
        self._token = token or os.environ.get("GOOGLE_OAUTH_ACCESS_TOKEN")
        self.http = session or requests.Session()

    def _headers(self) -> Dict[str, str]:
        if self._token is None and "googleapis.com" in self.endpoint:
            r = self.http.get("http://metadata.google.internal/computeMetadata/v1/instance/service-accounts/default/token",
                              headers={"Metadata-Flavor": "Google"}, timeout=5)
            self._token = _check(r, "gcs token").json()["access_token"]
        return {"Authorization": f"Bearer {self._token}"} if self._token else {}

    def _obj(self, key: str) -> str:
        return f"{self.endpoint}/storage/v1/b/{self.bucket}/o/{urllib.parse.quote(key, safe='')}"

    def put(self, key: str, path: str) -> None:
        url = f"{self.endpoint}/upload/storage/v1/b/{self.bucket}/o"
        with open(path, "rb") as f:
            _check(self.http.post(url, params={"uploadType": "media", "name": key}, data=f,
                                  headers=self._headers()), f"gcs put {key}")

    def get(self, key: str, path: str) -> None:
        _stream_to(_check(self.http.get(self._obj(key), params={"alt": "media"}, headers=self._headers(),
                                        stream=True), f"gcs get {key}"), path)

    def list(self, prefix: str) -> List[Tuple[str, int]]:
        out: List[Tuple[str, int]] = []
        page = None
        while True:
            params = {"prefix": prefix}
            if page:
                params["pageToken"] = page
            d = _check(self.http.get(f"{self.endpoint}/storage/v1/b/{self.bucket}/o", params=params,
                                     headers=self._headers()), "gcs list").json()
            out += [(o["name"], int(o.get("size", 0))) for o in d.get("items", [])]
            page = d.get("nextPageToken")
            if not page:
                return out

    def delete(self, key: str) -> None:
        _check(self.http.delete(self._obj(key), headers=self._headers()), f"gcs delete {key}")
