"""Infrastructure providers (the L0 substrate).

The reference talks to Joyent Triton through the ``triton`` CLI (setup.sh:210,257,259,536,541)
and the Terraform ``triton`` provider (terraform/master/main.tf:1). Providers here expose the
same four things behind one interface:

* ``env()``       — account credentials (``triton env`` → SDC_URL/SDC_ACCOUNT/SDC_KEY_ID)
* ``networks()``  — named networks with ids (``triton networks -oname,id``)
* ``packages()``  — machine shapes with ids (``triton packages -oname,id | grep -kvm-``)
* machine lifecycle: ``create_machine``/``exec``/``delete_machine`` (``triton_machine``)

``local`` (default) provisions worker sandboxes on this MI355X host; ``baremetal`` claims slices
of real hosts from an SSH inventory and configures them over SSH; ``triton`` shells out to the
real CLI for parity with the reference (untestable offline) and configures its VMs over SSH.
"""
from __future__ import annotations

from .base import Machine, Network, Package, Provider  # noqa: F401


def get_provider(name: str, state_dir, **kw) -> "Provider":
    if name == "local":
        from .local import LocalProvider

        return LocalProvider(state_dir, **kw)
    if name == "baremetal":
        from .baremetal import BareMetalProvider

        return BareMetalProvider(state_dir, **kw)
    if name == "triton":
        from .triton import TritonProvider

        return TritonProvider(state_dir, **kw)
    raise ValueError(f"unknown backend {name!r} (expected 'local', 'baremetal' or 'triton')")
