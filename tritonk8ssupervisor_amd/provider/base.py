"""Provider interface and value types."""
from __future__ import annotations

import abc

from ..utils.record import asdict, field, record as dataclass


@dataclass(frozen=True)
class Network:
    name: str
    id: str
    subnet: str = ""
    public: bool = False


@dataclass(frozen=True)
class Package:
    name: str
    id: str
    gpus: int = 0
    cpus: int = 0
    memory_mb: int = 0
    description: str = ""


@dataclass
class Machine:
    name: str
    id: str
    package: str
    networks: list[str]
    primaryip: str
    ips: list[str] = field(default_factory=list)
    gpus: list[int] = field(default_factory=list)  # host GPU ordinals owned by this machine
    image: str = ""
    tags: dict = field(default_factory=dict)
    sandbox: str = ""      # the machine's work dir (on the machine: remote path for remote providers)
    state: str = "running"
    home: str = ""         # tk8s install root on the machine ("" = the controller's own checkout)
    python: str = ""       # interpreter on the machine ("" = the controller's sys.executable)

    def to_dict(self) -> dict:
        return asdict(self)

    @classmethod
    def from_dict(cls, d: dict) -> "Machine":
        return cls(**{k: d[k] for k in (f.name for f in cls.__record_fields__) if k in d})


class ProvisionError(RuntimeError):
    pass


class Provider(abc.ABC):
    name = "abstract"
    default_network = ""
    default_package = ""
    # True when machines are sandboxes of the controller host (local provider): the orchestrator
    # may then spawn their daemons directly and run its boot hooks; otherwise every action goes
    # through exec() (ssh) -- executor.RemoteExecutor.
    colocated = False

    @abc.abstractmethod
    def env(self) -> dict[str, str]:
        """Credentials like `triton env`: SDC_URL, SDC_ACCOUNT, SDC_KEY_ID."""

    @abc.abstractmethod
    def networks(self) -> list[Network]:
        """Networks sorted by name (setup.sh:257 sorts `triton networks` output)."""

    @abc.abstractmethod
    def packages(self) -> list[Package]:
        """Machine shapes sorted by name (setup.sh:259)."""

    @abc.abstractmethod
    def find_key(self, key_id: str) -> str | None:
        """Private key path whose fingerprint is key_id (setup.sh:215-230), or None."""

    @abc.abstractmethod
    def create_machine(self, name: str, package: str, networks: list[str], image: str = "",
                       root_authorized_keys: str = "", tags: dict | None = None) -> Machine:
        ...

    @abc.abstractmethod
    def exec(self, machine: Machine, command: str, timeout: float = 300, env: dict | None = None,
             stdin: bytes | None = None) -> tuple[int, str]:
        """Run a shell command on the machine (remote-exec), in its work dir with its machine
        environment (TK8S_MACHINE*) plus ``env``; returns (rc, stdout+stderr)."""

    @abc.abstractmethod
    def delete_machine(self, machine: Machine) -> None:
        ...

    def get_machine(self, name: str) -> Machine | None:  # pragma: no cover - optional
        return None

    # ---- index helpers (getNetworkIDs / getPackageID, setup.sh:532-542) -------------
    def network_ids(self, indices: list[int]) -> list[str]:
        nets = self.networks()
        return [nets[i - 1].id for i in indices]

    def package_id(self, index: int) -> str:
        return self.packages()[index - 1].id

    def package_by_id_or_name(self, key: str) -> Package:
        for p in self.packages():
            if key in (p.id, p.name):
                return p
        raise ProvisionError(f"unknown package {key!r}")

    def network_by_id_or_name(self, key: str) -> Network:
        for n in self.networks():
            if key in (n.id, n.name):
                return n
        raise ProvisionError(f"unknown network {key!r}")
