"""The sidecar's network plugin and the SDK's network client, restated over the simulator.

Reference interfaces mirrored here:

* ``sidecar.Network`` (``pkg/sidecar/instance.go:37-42``): ``ConfigureNetwork(ctx, cfg)``,
  ``ListActive()``, ``Close()``. :class:`SimNetwork` implements it for one simulated instance by
  calling ``tgsim_configure_network_order`` (the docker apply order of
  ``pkg/sidecar/docker_network.go:51-148`` or the k8s one of ``pkg/sidecar/k8s_network.go:43-176``
  is inside the C ABI; the sidecar picks it by runner name like ``sidecar_linux.go:20-58``).
* The sidecar instance handler (``pkg/sidecar/sidecar_handler.go:15-83``): initial
  ``Config{Network: "default", Enable: true}``, ``SignalAndWait("network-initialized", N)``, then
  every published Config is applied in order and ``SignalEntry(cfg.CallbackState)`` follows when
  the callback state is set. :class:`Sidecar` runs that sequence for all instances at once.
* ``network.Client`` from sdk-go [EXT] (behaviour pinned by ``pkg/sidecar/sidecar_test.go:35``,
  ``:58-59``, ``:88-92``): an empty ``CallbackState`` is an error with the SDK's exact message;
  otherwise the config reaches the sidecar unmodified and the plan waits on
  ``Barrier(CallbackState, CallbackTarget or N)``. :class:`NetClient` mirrors it.

Configuration takes effect from the next simulated window for every message that window
processes.

``wire=True`` routes every config the way the reference does: ``NetClient`` publishes its JSON form
(``Config.to_wire``) on the sync topic ``network:<hostname>`` (device-resident topics)
and the instance's sidecar replays the topic from its last position, decodes each entry
(``Config.from_wire``) and applies it (``sidecar_handler.go:49-80``).
"""
from __future__ import annotations

import copy

import numpy as np

from . import _abi as A
from .network import Config
from .sync import SyncService

DEFAULT_DATA_NETWORK = "default"          # sidecar_handler.go:11-13
NET_INIT_STATE = "network-initialized"    # sidecar_handler.go:40
ERR_NO_CALLBACK = "failed to configure network; no callback state provided"  # sidecar_test.go:59


class SimNetwork:
    """sidecar.Network for one simulated instance."""

    def __init__(self, sim, instance: int, order: str = "docker"):
        self.sim = sim
        self.instance = int(instance)
        self.order = order
        self.active: dict[str, Config] = {}
        self.configured: list[Config] = []   # like MockNetwork.Configured (mock.go:72-76)
        self.closed = False

    def configure_network(self, cfg: Config) -> None:
        if self.closed:
            raise A.TgsimError(A.ESTATE, "network is closed")
        self.sim.configure(self.instance, cfg, self.order)
        self.configured.append(cfg)
        self.active[cfg.network] = cfg

    def list_active(self) -> list[str]:
        return [k for k, v in self.active.items() if v.enable]

    def close(self) -> None:
        self.closed = True


class Sidecar:
    """The per-instance sidecar handlers of one run, driven in lock step."""

    def __init__(self, sim, sync: SyncService, n_instances: int, track_configs: bool = False,
                 runner: str = "docker", wire: bool = False):
        if runner not in ("docker", "k8s"):
            raise ValueError(f"unknown sidecar runner {runner!r}")
        self.wire = wire
        self._consumed: dict[int, int] = {}   # wire mode: topic entries each sidecar has applied
        self.sim = sim
        self.order = runner
        self.sync = sync
        self.n = n_instances
        self.track = track_configs
        self._nets: dict[int, SimNetwork] = {}
        self.t_initialized = None

    def network(self, instance: int) -> SimNetwork:
        if instance not in self._nets:
            self._nets[instance] = SimNetwork(self.sim, instance, self.order)
        return self._nets[instance]

    def initialize(self, t: int = 0) -> int:
        """sidecar_handler.go:26-46 for every instance. The simulator's instances are created in
        the state the initial Config leaves them in; this records that config and runs
        SignalAndWait("network-initialized", N). Returns the release time."""
        init = Config(network=DEFAULT_DATA_NETWORK, enable=True)
        if self.track:
            for g in range(self.n):
                net = self.network(g)
                net.configured.append(init)
                net.active[DEFAULT_DATA_NETWORK] = init
        _, rel = self.sync.signal_and_wait(NET_INIT_STATE, np.arange(self.n), t, self.n)
        self.t_initialized = rel
        return rel

    @staticmethod
    def topic(instance: int) -> str:
        """The instance's config topic, "network:" + its hostname (sidecar_handler.go:49)."""
        return f"network:instance-{instance}"

    def poll(self, instance: int, t: int) -> int:
        """Wire mode: the instance's sidecar receives the configs published on its topic since its
        last poll, in topic order, and applies each one. Returns how many it applied."""
        entries = self.sync.subscribe(self.topic(instance), until_t=t)
        start = self._consumed.get(instance, 0)
        for d in entries[start:]:
            self.apply(instance, Config.from_wire(d), t)
        self._consumed[instance] = len(entries)
        return len(entries) - start

    def apply(self, instance: int, cfg: Config, t: int) -> None:
        """One iteration of the handler loop (sidecar_handler.go:64-80)."""
        if self.track:
            self.network(instance).configure_network(cfg)
        else:
            self.sim.configure(instance, cfg, self.order)
        if cfg.callback_state:
            self.sync.signal_entry(cfg.callback_state, [instance], t)


class NetClient:
    """network.Client of sdk-go [EXT] for simulated instances."""

    def __init__(self, sidecar: Sidecar):
        self.sidecar = sidecar

    def wait_network_initialized(self, t: int = 0) -> int:
        rel = self.sidecar.sync.barrier(NET_INIT_STATE, self.sidecar.n, t)
        if rel < 0:
            raise A.TgsimError(A.ESTATE, "network not initialized: the sidecar has not run")
        return rel

    def configure_network(self, instance: int, cfg: Config, t: int) -> int:
        """Publish cfg to the instance's sidecar and wait on Barrier(CallbackState, target).
        Returns the barrier release time (-1 while fewer than target sidecars have signalled)."""
        if not cfg.callback_state:
            raise ValueError(ERR_NO_CALLBACK)
        if self.sidecar.wire:   # publish on network:<hostname>; the sidecar's subscription applies it
            self.sidecar.sync.publish(Sidecar.topic(instance), [instance], t, [cfg.to_wire()])
            self.sidecar.poll(instance, t)
        else:
            # the plan may change its Config after the call (pingpong.go mutates latency and IP):
            # the sidecar keeps a copy; rule lists are shared, not copied (plans never edit one in
            # place, and a shared RuleList keeps its C array)
            c = copy.copy(cfg)
            c.default = copy.copy(cfg.default)
            self.sidecar.apply(instance, c, t)
        target = cfg.callback_target or self.sidecar.n
        return self.sidecar.sync.barrier(cfg.callback_state, target, t)

    def get_data_network_ip(self, instance: int) -> int:
        return self.sidecar.sim.get_ip(instance)
