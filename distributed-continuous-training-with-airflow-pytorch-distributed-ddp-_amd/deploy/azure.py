"""Azure ML online-endpoint deployment and the blue/green -> shadow -> canary -> full rollout.

Reference behaviour:
  * ``force_deploy`` (dags/azure_manual_deploy.py:137-167): get the endpoint; if missing or in a
    failed provisioning state, (delete and) create it with ``auth_mode="key"``; create/update
    deployment ``DEPLOYMENT_NAME`` (Standard_DS2_v2 x 1, openmpi4.1.0-ubuntu20.04 + conda.yaml);
    send 100 % of the traffic to it.
  * automated rollout (dags/azure_auto_deploy.py:118-185): new slot = ``blue`` if the endpoint
    has no traffic, else the opposite of the slot holding the most traffic; deploy it; shadow
    (``traffic {old:100,new:0}``, ``mirror_traffic {new:20}``); wait; canary
    (``{old:90,new:10}``, no mirror); wait; full (``{new:100}``) and delete the old deployment.
Fixes kept deliberately: the config is read correctly (reference D1 assigned every value to one
variable), and each phase can be gated by a health probe with automatic rollback to the old
slot (reference D11 only slept).  The Azure SDK (``azure-ai-ml``) is imported lazily; tests and
dry runs inject :class:`FakeMLClient`, which models endpoints, deployments and traffic maps.
"""
from __future__ import annotations

import copy
import logging
import os
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, Optional

log = logging.getLogger(__name__)

DEFAULT_IMAGE = "mcr.microsoft.com/azureml/openmpi4.1.0-ubuntu20.04"
DEFAULT_INSTANCE = "Standard_DS2_v2"


@dataclass
class AzureConfig:
    subscription_id: Optional[str] = None
    resource_group: Optional[str] = None
    workspace: Optional[str] = None
    endpoint_name: Optional[str] = None
    deploy_dir: Optional[str] = None
    deployment_name: str = "blue"
    instance_type: str = DEFAULT_INSTANCE
    instance_count: int = 1
    image: str = DEFAULT_IMAGE
    shadow_mirror_pct: int = 20
    canary_pct: int = 10
    wait_s: float = 30.0

    @classmethod
    def from_env(cls, env=None) -> "AzureConfig":
        e = os.environ if env is None else env
        return cls(subscription_id=e.get("AZURE_SUBSCRIPTION_ID"), resource_group=e.get("AZURE_RESOURCE_GROUP"),
                   workspace=e.get("AZURE_WORKSPACE"), endpoint_name=e.get("ENDPOINT_NAME"),
                   deploy_dir=e.get("DEPLOY_DIR"), deployment_name=e.get("DEPLOYMENT_NAME", "blue"))


# ----------------------------------------------------------------------------- entities
def _entities():
    """(ManagedOnlineEndpoint, ManagedOnlineDeployment, Model, Environment, CodeConfiguration)."""
    try:
        from azure.ai.ml.entities import (CodeConfiguration, Environment, ManagedOnlineDeployment,
                                          ManagedOnlineEndpoint, Model)

        return ManagedOnlineEndpoint, ManagedOnlineDeployment, Model, Environment, CodeConfiguration
    except Exception:  # noqa: BLE001 - SDK absent: light stand-ins with the same fields
        return _Endpoint, _Deployment, _Model, _Environment, _CodeConfiguration


@dataclass
class _Endpoint:
    name: str
    auth_mode: str = "key"
    traffic: Dict[str, int] = field(default_factory=dict)
    mirror_traffic: Dict[str, int] = field(default_factory=dict)
    provisioning_state: str = "Succeeded"


@dataclass
class _Model:
    path: str


@dataclass
class _Environment:
    conda_file: str
    image: str


@dataclass
class _CodeConfiguration:
    code: str
    scoring_script: str


@dataclass
class _Deployment:
    name: str
    endpoint_name: str
    model: _Model = None
    code_configuration: _CodeConfiguration = None
    environment: _Environment = None
    instance_type: str = DEFAULT_INSTANCE
    instance_count: int = 1
    provisioning_state: str = "Succeeded"


def get_ml_client(cfg: AzureConfig):
    from azure.ai.ml import MLClient
    from azure.identity import DefaultAzureCredential

    return MLClient(DefaultAzureCredential(), cfg.subscription_id, cfg.resource_group, cfg.workspace)


def _build_deployment(cfg: AzureConfig, name: str):
    _, Deployment, Model, Environment, CodeConfiguration = _entities()
    d = cfg.deploy_dir
    return Deployment(
        name=name,
        endpoint_name=cfg.endpoint_name,
        model=Model(path=d),
        code_configuration=CodeConfiguration(code=d, scoring_script="score.py"),
        environment=Environment(conda_file=os.path.join(d, "conda.yaml"), image=cfg.image),
        instance_type=cfg.instance_type,
        instance_count=cfg.instance_count,
    )


# ----------------------------------------------------------------------------- manual / forced
def ensure_endpoint(client, cfg: AzureConfig):
    """Get the endpoint, (re)creating it (key auth) when missing or in a failed state."""
    Endpoint = _entities()[0]
    endpoint = None
    try:
        endpoint = client.online_endpoints.get(name=cfg.endpoint_name)
        if str(getattr(endpoint, "provisioning_state", "")).lower() == "failed":
            log.warning("endpoint %s is in a failed state; recreating", cfg.endpoint_name)
            client.online_endpoints.begin_delete(name=cfg.endpoint_name).wait()
            endpoint = None
    except Exception:  # noqa: BLE001 - not found
        endpoint = None
    if endpoint is None:
        endpoint = Endpoint(name=cfg.endpoint_name, auth_mode="key")
        client.online_endpoints.begin_create_or_update(endpoint).result()
        endpoint = client.online_endpoints.get(name=cfg.endpoint_name)
    return endpoint


def force_deploy(client, cfg: AzureConfig) -> str:
    ensure_endpoint(client, cfg)
    client.online_deployments.begin_create_or_update(_build_deployment(cfg, cfg.deployment_name)).result()
    endpoint = client.online_endpoints.get(name=cfg.endpoint_name)
    endpoint.traffic = {cfg.deployment_name: 100}
    client.online_endpoints.begin_create_or_update(endpoint).result()
    return cfg.deployment_name


# ----------------------------------------------------------------------------- blue/green rollout
def choose_slots(traffic: Optional[Dict[str, int]]):
    """(old_slot, new_slot): blue when nothing is live, else the other colour of the live max."""
    if not traffic or sum(traffic.values()) == 0:
        return "blue", "blue"
    current = max(traffic, key=traffic.get)
    return current, ("green" if current == "blue" else "blue")


def deploy_new_slot(client, cfg: AzureConfig) -> Dict[str, str]:
    endpoint = ensure_endpoint(client, cfg)  # the reference required a pre-existing endpoint
    old, new = choose_slots(getattr(endpoint, "traffic", None))
    log.info("live slot %s; deploying %s", old, new)
    client.online_deployments.begin_create_or_update(_build_deployment(cfg, new)).result()
    return {"old_slot": old, "new_slot": new}


def set_traffic(client, cfg: AzureConfig, traffic: Dict[str, int], mirror: Optional[Dict[str, int]] = None):
    endpoint = client.online_endpoints.get(name=cfg.endpoint_name)
    endpoint.traffic = dict(traffic)
    endpoint.mirror_traffic = dict(mirror or {})
    client.online_endpoints.begin_create_or_update(endpoint).result()


def start_shadow(client, cfg: AzureConfig, old: str, new: str):
    if new == old:
        return
    set_traffic(client, cfg, {old: 100, new: 0}, {new: cfg.shadow_mirror_pct})


def start_canary(client, cfg: AzureConfig, old: str, new: str):
    if new == old:
        return
    set_traffic(client, cfg, {old: 100 - cfg.canary_pct, new: cfg.canary_pct}, {})


def full_rollout(client, cfg: AzureConfig, old: str, new: str):
    set_traffic(client, cfg, {new: 100}, {})
    if new != old:
        log.info("deleting old deployment %s", old)
        client.online_deployments.begin_delete(name=old, endpoint_name=cfg.endpoint_name).wait()


def rollback(client, cfg: AzureConfig, old: str, new: str):
    """Send everything back to the old slot and remove the new deployment (health gate failed)."""
    if new == old:
        return
    set_traffic(client, cfg, {old: 100}, {})
    client.online_deployments.begin_delete(name=new, endpoint_name=cfg.endpoint_name).wait()


def automated_rollout(client, cfg: AzureConfig, probe: Optional[Callable[[str], bool]] = None,
                      sleep: Callable[[float], None] = time.sleep) -> Dict[str, str]:
    """deploy_new_slot -> shadow -> wait -> canary -> wait -> full, gated by ``probe(slot)``."""
    slots = deploy_new_slot(client, cfg)
    old, new = slots["old_slot"], slots["new_slot"]
    phases = [("shadow", start_shadow), ("canary", start_canary)]
    for name, fn in phases:
        fn(client, cfg, old, new)
        sleep(cfg.wait_s)
        if probe is not None and new != old and not probe(new):
            log.error("health gate failed during %s; rolling back to %s", name, old)
            rollback(client, cfg, old, new)
            return {**slots, "status": f"rolled_back_at_{name}"}
    full_rollout(client, cfg, old, new)
    return {**slots, "status": "complete"}


# ----------------------------------------------------------------------------- fake client
class _Poller:
    def __init__(self, result=None):
        self._r = result

    def result(self):
        return self._r

    def wait(self):
        return self._r


class FakeMLClient:
    """In-memory MLClient: endpoints with traffic/mirror maps, deployments, an operation log."""

    class _Endpoints:
        def __init__(self, outer):
            self.o = outer

        def get(self, name):
            if name not in self.o.endpoints:
                raise KeyError(f"endpoint {name} not found")
            return copy.deepcopy(self.o.endpoints[name])

        def begin_create_or_update(self, ep):
            for slot in list(getattr(ep, "traffic", {}) or {}) + list(getattr(ep, "mirror_traffic", {}) or {}):
                if (ep.traffic or {}).get(slot, 0) or (ep.mirror_traffic or {}).get(slot, 0):
                    if (ep.name, slot) not in self.o.deployments:
                        raise ValueError(f"traffic to unknown deployment {slot}")
            if sum((ep.traffic or {}).values()) not in (0, 100):
                raise ValueError("traffic must sum to 100")
            self.o.endpoints[ep.name] = copy.deepcopy(ep)
            self.o.log.append(("endpoint", ep.name, dict(ep.traffic or {}), dict(getattr(ep, "mirror_traffic", {}) or {})))
            return _Poller(ep)

        def begin_delete(self, name):
            self.o.endpoints.pop(name, None)
            self.o.log.append(("delete_endpoint", name))
            return _Poller()

    class _Deployments:
        def __init__(self, outer):
            self.o = outer

        def begin_create_or_update(self, d):
            if d.endpoint_name not in self.o.endpoints:
                raise ValueError("endpoint does not exist")
            self.o.deployments[(d.endpoint_name, d.name)] = d
            self.o.log.append(("deploy", d.name))
            return _Poller(d)

        def begin_delete(self, name, endpoint_name):
            self.o.deployments.pop((endpoint_name, name), None)
            self.o.log.append(("delete_deployment", name))
            return _Poller()

        def list(self, endpoint_name):
            return [d for (e, _), d in self.o.deployments.items() if e == endpoint_name]

    def __init__(self):
        self.endpoints: Dict[str, _Endpoint] = {}
        self.deployments: Dict[tuple, _Deployment] = {}
        self.log = []
        self.online_endpoints = FakeMLClient._Endpoints(self)
        self.online_deployments = FakeMLClient._Deployments(self)
