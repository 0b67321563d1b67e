"""KFModel -- the plugin base class (mirror of python/kfserving/kfserving/kfmodel.py:31-122).

Same constructor, attributes (name, ready, protocol, predictor_host,
explainer_host, timeout), and load / preprocess / postprocess / predict /
explain contract.  preprocess unwraps a binary-mode CloudEvent (kfmodel.py:58-70)
and a structured CloudEvent dict (kfmodel.py:75-81) as the reference does; predict/explain forward to ``predictor_host`` over HTTP
when set (kfmodel.py:88-122), otherwise raise NotImplementedError.
"""
from __future__ import annotations

import asyncio
import json
import urllib.error
import urllib.request
from typing import Dict

from .cloudevent import CloudEvent
from .errors import HTTPError

PREDICTOR_URL_FORMAT = "http://{0}/v1/models/{1}:predict"
EXPLAINER_URL_FORMAT = "http://{0}/v1/models/{1}:explain"
PREDICTOR_V2_URL_FORMAT = "http://{0}/v2/models/{1}/infer"
EXPLAINER_V2_URL_FORMAT = "http://{0}/v2/models/{1}/explain"

_CE_STRUCTURED_KEYS = ("time", "type", "source", "id", "specversion", "data")


class KFModel:
    def __init__(self, name: str):
        self.name = name
        self.ready = False
        self.protocol = "v1"
        self.predictor_host = None
        self.explainer_host = None
        # matches the timeout of the generated Istio resources (kfmodel.py:40-43)
        self.timeout = 600

    def load(self) -> bool:
        self.ready = True
        return self.ready

    def preprocess(self, request: Dict) -> Dict:
        # binary-mode CloudEvent (kfmodel.py:58-70): its data, JSON-decoded when
        # it is bytes; undecodable bytes are passed on, unless the event says
        # its content is JSON (400)
        if isinstance(request, CloudEvent):
            response = request.data
            if isinstance(response, bytes):
                try:
                    response = json.loads(response.decode("UTF-8"))
                except (json.JSONDecodeError, UnicodeDecodeError) as e:
                    if request._attributes.get("content-type") in (
                            "application/cloudevents+json", "application/json"):
                        raise HTTPError(400, "Unrecognized request format: %s" % e)
            return response
        # structured CloudEvent: {"time","type","source","id","specversion","data"}
        if isinstance(request, dict) and all(k in request for k in _CE_STRUCTURED_KEYS):
            return request["data"]
        return request

    def postprocess(self, request: Dict) -> Dict:
        return request

    async def _forward(self, url: str, request: Dict) -> Dict:
        body = json.dumps(request).encode()

        def call():
            req = urllib.request.Request(url, data=body, method="POST",
                                         headers={"Content-Type": "application/json"})
            try:
                with urllib.request.urlopen(req, timeout=self.timeout) as resp:
                    return resp.status, resp.read()
            except urllib.error.HTTPError as e:
                return e.code, e.read()

        code, payload = await asyncio.get_running_loop().run_in_executor(None, call)
        if code != 200:
            raise HTTPError(code, payload.decode("utf-8", "replace"))
        return json.loads(payload)

    async def predict(self, request: Dict) -> Dict:
        if not self.predictor_host:
            raise NotImplementedError
        fmt = PREDICTOR_V2_URL_FORMAT if self.protocol == "v2" else PREDICTOR_URL_FORMAT
        return await self._forward(fmt.format(self.predictor_host, self.name), request)

    async def explain(self, request: Dict) -> Dict:
        if self.explainer_host is None:
            raise NotImplementedError
        fmt = EXPLAINER_V2_URL_FORMAT if self.protocol == "v2" else EXPLAINER_URL_FORMAT
        # the reference formats the explainer URL with predictor_host (kfmodel.py:109-111)
        return await self._forward(fmt.format(self.predictor_host, self.name), request)
