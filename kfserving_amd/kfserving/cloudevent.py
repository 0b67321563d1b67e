"""CloudEvents (spec 1.0) in binary content mode over HTTP, for ``:predict``.

The reference decodes and re-encodes them with the ``cloudevents`` SDK
(python/kfserving/kfserving/handlers/http.py:55-66 and :81-91; KFModel.preprocess
kfmodel.py:58-70).  Binary mode is plain HTTP: the event's attributes travel as
``ce-<name>`` headers, ``datacontenttype`` as ``Content-Type``, the data as the
body, so this module needs no SDK (it is not installed here).  What it keeps
from the reference's use of the SDK:

* a request is a binary event when it carries ``ce-specversion``,
  ``ce-source``, ``ce-type`` and ``ce-id`` (``has_binary_headers``);
* attributes = the ``ce-*`` headers without the prefix, plus ``datacontenttype``
  from ``Content-Type``; ``specversion`` must be ``1.0`` or ``0.3``;
* the data stays the raw body bytes unless the request has a ``ce-contenttype``
  header, in which case it is JSON-decoded when it decodes (the SDK's default
  unmarshaller);
* the response is an event with the request's attributes and the model's
  response as data, written back in binary mode: ``ce-<name>`` for every
  attribute, ``Content-Type`` = ``datacontenttype``, ``ce-time`` = the current
  UTC time as ``%Y-%m-%dT%H:%M:%S.%f%z``, body = ``json.dumps`` of the response
  (test_server.py:262-303 asserts these bytes and headers).
"""
from __future__ import annotations

import json
from datetime import datetime, timezone
from typing import Any, Dict, Mapping, Tuple

_REQUIRED = ("ce-specversion", "ce-source", "ce-type", "ce-id")
_VERSIONS = ("1.0", "0.3")


class CloudEventError(ValueError):
    """Malformed binary-mode event (the SDK's MissingRequiredFields /
    InvalidRequiredFields family); KFServer answers 400."""


class CloudEvent:
    """Attributes + data of one event (the reference's ``body._attributes``)."""

    def __init__(self, attributes: Dict[str, str], data: Any):
        self._attributes = dict(attributes)
        self.data = data

    def __getitem__(self, key):
        return self._attributes[key]


def has_binary_headers(headers: Mapping[str, str]) -> bool:
    """``headers`` keys are lower case (kfserver._read_request)."""
    return all(h in headers for h in _REQUIRED)


def from_binary_http(headers: Mapping[str, str], body: bytes) -> CloudEvent:
    attrs = {k[3:]: v for k, v in headers.items() if k.startswith("ce-")}
    if "content-type" in headers:
        attrs["datacontenttype"] = headers["content-type"]
    for req in ("specversion", "source", "type", "id"):
        if not attrs.get(req):
            raise CloudEventError(f"Missing required attribute: {req}")
    if attrs["specversion"] not in _VERSIONS:
        raise CloudEventError(f"Found invalid specversion {attrs['specversion']}")
    data: Any = body
    if "ce-contenttype" in headers:      # the SDK's default data unmarshaller
        try:
            data = json.loads(body)
        except (json.JSONDecodeError, TypeError, UnicodeDecodeError):
            data = body
    return CloudEvent(attrs, data)


def utc_now() -> str:
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%f%z")


def to_binary_http(event: CloudEvent, response: Any) -> Tuple[Dict[str, str], bytes]:
    """Headers and body of the response event (request attributes, model
    response as data), ``ce-time`` set to now as the reference handler does."""
    headers: Dict[str, str] = {}
    ct = event._attributes.get("datacontenttype")
    if ct is not None:
        headers["Content-Type"] = ct
    for k, v in event._attributes.items():
        headers["ce-" + k] = utc_now() if k == "time" else str(v)
    if "time" not in event._attributes:
        headers["ce-time"] = utc_now()
    if isinstance(response, (bytes, bytearray)):
        body = bytes(response)
    elif isinstance(response, str):
        body = response.encode("utf-8")
    else:
        body = json.dumps(response).encode("utf-8")
    return headers, body
