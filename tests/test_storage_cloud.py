"""REST object-store checkpoint backends (common/storage/_cloud.py) against in-process fake S3,
Azure Blob and GCS servers that verify the request signatures; plus the published AWS SigV4
``get-vanilla`` test vector."""
import hashlib
import http.server
import json
import threading
import urllib.parse
import xml.sax.saxutils as sx

import pytest

from determined_clone_amd.common import storage
from determined_clone_amd.common.storage import _cloud
from determined_clone_amd.errors import CheckpointNotFoundException

AK, SK = "AKIDTEST", "secret/key+example"
AZ_ACCOUNT, AZ_KEY = "devacct", "c2VjcmV0LWF6dXJlLWtleS1mb3ItdGVzdHM="
GCS_TOKEN = "ya29.test-token"


def test_sigv4_matches_aws_test_suite_get_vanilla():
    h = _cloud.sigv4_headers("GET", "https://example.amazonaws.com/", {}, _cloud.EMPTY_SHA256,
                             "AKIDEXAMPLE", "wJalrXUtnFEMI/K7MDENG+bPxRfiCYEXAMPLEKEY", "us-east-1",
                             "service", amz_date="20150830T123600Z")
    assert h["Authorization"] == (
        "AWS4-HMAC-SHA256 Credential=AKIDEXAMPLE/20150830/us-east-1/service/aws4_request, "
        "SignedHeaders=host;x-amz-date, "
        "Signature=5fa00fa31553b73ebf1942676e86291e8372ff2a2260956d9b8aae1d763fbf31")


class _Fake(http.server.BaseHTTPRequestHandler):
    objects: dict = {}
    kind = "s3"
    page = 2

    def log_message(self, *a):
        pass

    def _body(self):
        n = int(self.headers.get("Content-Length") or 0)
        return self.rfile.read(n) if n else b""

    def _reply(self, code, body=b"", ctype="application/xml"):
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def _auth_ok(self, body):
        url = f"http://{self.headers['Host']}{self.path}"
        if self.kind == "s3":
            sha = self.headers.get("x-amz-content-sha256")
            if sha != hashlib.sha256(body).hexdigest():
                return False
            want = _cloud.sigv4_headers(self.command, url, {"x-amz-content-sha256": sha}, sha, AK, SK,
                                        "us-east-1", "s3", amz_date=self.headers["x-amz-date"])
            return want["Authorization"] == self.headers.get("Authorization")
        if self.kind == "azure":
            hdrs = {k: v for k, v in self.headers.items() if k.lower().startswith("x-ms-")
                    or k.lower() in ("content-length", "content-type")}
            return _cloud.azure_shared_key(self.command, url, hdrs, AZ_ACCOUNT, AZ_KEY) == self.headers.get("Authorization")
        return self.headers.get("Authorization") == f"Bearer {GCS_TOKEN}"

    def _handle(self):
        body = self._body()
        if not self._auth_ok(body):
            return self._reply(403, b"bad signature")
        u = urllib.parse.urlsplit(self.path)
        q = dict(urllib.parse.parse_qsl(u.query))
        if self.kind == "gcs":
            return self._gcs(u, q, body)
        parts = urllib.parse.unquote(u.path).lstrip("/").split("/", 1)
        key = parts[1] if len(parts) > 1 else ""
        listing = (self.kind == "s3" and q.get("list-type") == "2") or (self.kind == "azure" and q.get("comp") == "list")
        if self.command == "GET" and listing:
            keys = sorted(k for k in self.objects if k.startswith(q.get("prefix", "")))
            start = int(q.get("continuation-token") or q.get("marker") or 0)
            chunk, nxt = keys[start:start + self.page], start + self.page
            more = nxt < len(keys)
            if self.kind == "s3":
                items = "".join(f"<Contents><Key>{sx.escape(k)}</Key><Size>{len(self.objects[k])}</Size></Contents>" for k in chunk)
                xml = (f'<ListBucketResult xmlns="http://s3.amazonaws.com/doc/2006-03-01/">{items}'
                       f"<IsTruncated>{'true' if more else 'false'}</IsTruncated>"
                       + (f"<NextContinuationToken>{nxt}</NextContinuationToken>" if more else "") + "</ListBucketResult>")
            else:
                items = "".join(f"<Blob><Name>{sx.escape(k)}</Name><Properties><Content-Length>{len(self.objects[k])}"
                                f"</Content-Length></Properties></Blob>" for k in chunk)
                xml = f"<EnumerationResults><Blobs>{items}</Blobs><NextMarker>{nxt if more else ''}</NextMarker></EnumerationResults>"
            return self._reply(200, xml.encode())
        if self.command == "PUT":
            if self.kind == "azure" and self.headers.get("x-ms-blob-type") != "BlockBlob":
                return self._reply(400)
            self.objects[key] = body
            return self._reply(201 if self.kind == "azure" else 200)
        if key not in self.objects:
            return self._reply(404)
        if self.command == "GET":
            return self._reply(200, self.objects[key], "application/octet-stream")
        if self.command == "DELETE":
            del self.objects[key]
            return self._reply(202 if self.kind == "azure" else 204)
        return self._reply(405)

    def _gcs(self, u, q, body):
        p = urllib.parse.unquote(u.path)
        if self.command == "POST" and p.startswith("/upload/storage/v1/b/"):
            self.objects[q["name"]] = body
            return self._reply(200, b"{}", "application/json")
        if p.endswith("/o") and self.command == "GET":
            keys = sorted(k for k in self.objects if k.startswith(q.get("prefix", "")))
            start = int(q.get("pageToken") or 0)
            d = {"items": [{"name": k, "size": str(len(self.objects[k]))} for k in keys[start:start + self.page]]}
            if start + self.page < len(keys):
                d["nextPageToken"] = str(start + self.page)
            return self._reply(200, json.dumps(d).encode(), "application/json")
        key = p.split("/o/", 1)[1]
        if key not in self.objects:
            return self._reply(404)
        if self.command == "GET":
            return self._reply(200, self.objects[key], "application/octet-stream")
        del self.objects[key]
        return self._reply(204)

    do_GET = do_PUT = do_DELETE = do_POST = _handle


@pytest.fixture(params=["s3", "azure", "gcs"])
def backend(request):
    handler = type("H", (_Fake,), {"objects": {}, "kind": request.param})
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), handler)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    url = f"http://127.0.0.1:{srv.server_address[1]}"
    if request.param == "s3":
        sm = storage.build({"type": "s3", "bucket": "ckpts", "access_key": AK, "secret_key": SK,
                            "endpoint_url": url, "prefix": "runs/a"})
    elif request.param == "azure":
        cs = f"AccountName={AZ_ACCOUNT};AccountKey={AZ_KEY};BlobEndpoint={url}"
        sm = storage.build({"type": "azure", "container": "ckpts", "connection_string": cs, "prefix": "runs/a"})
    else:
        sm = storage.GCSStorageManager("ckpts", prefix="runs/a", endpoint_url=url)
        sm.store._token = GCS_TOKEN
    yield sm, handler
    srv.shutdown()


def test_object_store_checkpoint_round_trip(backend, tmp_path):
    sm, handler = backend
    with sm.store_path("uuid-1") as p:
        (p / "state_dict.pth").write_bytes(b"weights" * 100)
        (p / "load_data.json").write_text("{}")
        (p / "sub").mkdir()
        (p / "sub" / "a b.txt").write_text("space in name")
    assert any(k.endswith("uuid-1/sub/a b.txt") for k in handler.objects)
    assert all(k.startswith("runs/a/uuid-1/") or "/uuid-1/" in k for k in handler.objects)
    files = sm.list_files("uuid-1")
    assert files == {"state_dict.pth": 700, "load_data.json": 2, "sub/a b.txt": 13}
    with sm.restore_path("uuid-1", selector=lambda rel: not rel.endswith(".pth")) as r:
        assert (r / "sub" / "a b.txt").read_text() == "space in name"
        assert not (r / "state_dict.pth").exists()
    left = sm.delete("uuid-1", ["*.pth"])
    assert set(left) == {"load_data.json", "sub/a b.txt"}
    sm.delete("uuid-1")
    assert sm.list_files("uuid-1") == {}
    with pytest.raises(CheckpointNotFoundException):
        sm.download("uuid-1", str(tmp_path / "x"))


def test_bad_credentials_are_rejected(tmp_path):
    handler = type("H", (_Fake,), {"objects": {}, "kind": "s3"})
    srv = http.server.ThreadingHTTPServer(("127.0.0.1", 0), handler)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        sm = storage.S3StorageManager("b", AK, "wrong", f"http://127.0.0.1:{srv.server_address[1]}")
        (tmp_path / "f").write_text("x")
        with pytest.raises(RuntimeError, match="403"):
            sm.upload(str(tmp_path), "u")
    finally:
        srv.shutdown()


def test_tensorboard_fetcher_syncs_event_files_from_object_storage(backend, tmp_path, monkeypatch):
    """Trial side: TensorboardManager uploads event files to the object store; TB task side: the
    fetcher pulls new / grown files and the task serves their scalars and images (reference
    tensorboard/fetchers/{s3,gcs,azure}.py, exec/tensorboard.py)."""
    import urllib.request

    from determined_clone_amd import tensorboard
    from determined_clone_amd.exec import tensorboard as tb_task
    from determined_clone_amd.tensorboard import fetchers

    sm, handler = backend
    base = tmp_path / "trial-tb"
    rel = "tensorboard/c1/experiment/7/trial/3"
    mgr = tensorboard.TensorboardManager(base, None, sm, rel)
    w = mgr.metric_writer()
    w.on_metrics("training", 1, {"loss": 0.5})
    png = b"\x89PNG\r\n\x1a\nfakepng"
    w._w._write(tensorboard.encode_image_event("samples", png, 2, 3, step=1))
    w._w.flush()
    mgr.sync()
    assert any("tensorboard/c1/experiment/7/trial/3/" in k for k in handler.objects)
    local = tmp_path / "tb-local"
    f = fetchers.build({"type": "s3"}, ["tensorboard/c1/experiment/7"], str(local), manager=sm)
    assert f.fetch_new() == 1
    assert f.fetch_new() == 0  # nothing changed
    w.on_metrics("training", 2, {"loss": 0.25})
    w._w.flush()
    mgr.sync()
    assert f.fetch_new() == 1  # the grown event file again
    logdir = str(local / "tensorboard/c1/experiment/7")
    runs = tensorboard.read_scalars(logdir)
    (run, tags), = runs.items()
    assert run == "trial/3" and [s for s, _, _ in next(iter(tags.values()))] == [1, 2]
    srv = tb_task.make_server({"exp7": logdir}, host="127.0.0.1")
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    url = f"http://127.0.0.1:{srv.server_address[1]}"
    meta = json.load(urllib.request.urlopen(f"{url}/data/images?run=exp7/trial/3&tag=samples"))
    assert meta[0]["height"] == 2 and meta[0]["width"] == 3 and meta[0]["step"] == 1
    assert urllib.request.urlopen(f"{url}/data/image?run=exp7/trial/3&tag=samples&index=0").read() == png
    assert b"<img" in urllib.request.urlopen(url + "/").read()
    srv.shutdown()
