#!/usr/bin/python
# -*- coding: utf-8 -*-
"""Ansible module tk8s_burnin: Start the early GPU burn-in on this machine's MI355X GPUs (one-shot daemon, result shared with the validation pod).

Real-Ansible front end of the in-repo playbook engine's module of the same name: it runs on the
target machine, finds that machine's tk8s install ($TK8S_HOME, or the newest ~/.tk8s/dist/<digest>
the baremetal/triton providers push) and calls the shared implementation
(tritonk8ssupervisor_amd/ansible_bridge.py -> playbook_modules.py). Arguments: ansible_bridge.ARG_SPECS.
"""
import glob
import os
import sys

DOCUMENTATION = r"""
module: tk8s_burnin
short_description: Start the early GPU burn-in on this machine's MI355X GPUs (one-shot daemon, result shared with the validation pod)
description: see tritonk8ssupervisor_amd/ansible_bridge.py (ARG_SPECS) and playbook_modules.py
"""


def _home():
    cands = [os.environ.get("TK8S_HOME", "")]
    cands += sorted(glob.glob(os.path.expanduser("~/.tk8s/dist/*")), key=os.path.getmtime, reverse=True)
    for c in cands:
        if c and os.path.isdir(os.path.join(c, "tritonk8ssupervisor_amd")):
            return c
    return None


if __name__ == "__main__":
    home = _home()
    if home and home not in sys.path:
        sys.path.insert(0, home)
    from tritonk8ssupervisor_amd.ansible_bridge import main

    main("tk8s_burnin")
