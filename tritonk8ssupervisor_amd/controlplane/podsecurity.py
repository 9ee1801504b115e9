"""Pod Security admission: the namespace labels ``pod-security.kubernetes.io/enforce`` and
``pod-security.kubernetes.io/warn`` (``privileged`` | ``baseline`` | ``restricted``) select the
Pod Security Standards a pod of that namespace must meet -- enforced (403) or warned about (a
``Warning`` header), as kube-apiserver's PodSecurity plugin does. Controllers' pods are checked
as well (their owner gets a FailedCreate event).

The checks are the standards' (v1.30) for what a pod spec can say here:

* baseline: no ``hostNetwork``/``hostPID``/``hostIPC``, no privileged containers, no
  ``hostPath`` volumes, no ``hostPort``s, capabilities added only from the default set, no
  ``Unconfined`` seccomp/AppArmor, ``procMount`` Default, no custom SELinux user/role;
* restricted: baseline plus volumes only of the ephemeral/projected kinds (configMap, secret,
  downwardAPI, emptyDir, projected, persistentVolumeClaim, ephemeral, csi), ``runAsNonRoot: true``
  and no ``runAsUser: 0``, ``allowPrivilegeEscalation: false``, capabilities dropping ``ALL``
  (adding at most ``NET_BIND_SERVICE``), a ``RuntimeDefault`` or ``Localhost`` seccomp profile.

What every pod gets whatever its level (the node's runtime, not this admission): the jail
(native/tools/gpujail.h) opens no render node of a GPU the pod does not hold, never creates a
device node (MAKE_CHAR / MAKE_BLOCK are handled and never granted) and denies the cluster's state
(the workspace's ``.tk8s/``: kubeconfig, tokens, keys, other pods' directories); image pods run
after ``pivot_root`` with Docker's default capability bounding set, the host's ``/sys`` and
``/proc/sys`` read-only (native/tools/tk8s_container.cpp). A multi-tenant GPU cluster adds
``baseline`` to keep tenants from ``hostPath`` volumes and the host's namespaces.
"""
from __future__ import annotations

LEVELS = ("privileged", "baseline", "restricted")
ENFORCE = "pod-security.kubernetes.io/enforce"
WARN = "pod-security.kubernetes.io/warn"
_BASELINE_CAPS = {"AUDIT_WRITE", "CHOWN", "DAC_OVERRIDE", "FOWNER", "FSETID", "KILL", "MKNOD", "NET_BIND_SERVICE",
                  "SETFCAP", "SETGID", "SETPCAP", "SETUID", "SYS_CHROOT"}
_RESTRICTED_VOLUMES = {"configMap", "secret", "downwardAPI", "emptyDir", "projected", "persistentVolumeClaim",
                       "ephemeral", "csi"}


def violations(pod: dict, level: str) -> list[str]:
    """What ``pod`` does that the ``level`` standard forbids (empty: it meets it)."""
    if level not in ("baseline", "restricted"):
        return []
    spec = pod.get("spec") or {}
    psc = spec.get("securityContext") or {}
    conts = (spec.get("containers") or []) + (spec.get("initContainers") or []) + (spec.get("ephemeralContainers") or [])
    out = []
    for f in ("hostNetwork", "hostPID", "hostIPC"):
        if spec.get(f):
            out.append(f"host namespaces ({f}=true)")
    priv = [c.get("name") for c in conts if (c.get("securityContext") or {}).get("privileged")]
    if priv:
        out.append(f"privileged (containers {', '.join(map(str, priv))} must not set securityContext.privileged=true)")
    hp = [v.get("name") for v in spec.get("volumes") or [] if "hostPath" in v]
    if hp:
        out.append(f"hostPath volumes (volumes {', '.join(map(str, hp))})")
    ports = [str(p.get("hostPort")) for c in conts for p in c.get("ports") or [] if p.get("hostPort")]
    if ports:
        out.append(f"hostPort (hostPorts {', '.join(ports)})")
    caps = {x for c in conts for x in ((c.get("securityContext") or {}).get("capabilities") or {}).get("add") or []}
    if caps - _BASELINE_CAPS:
        out.append(f"non-default capabilities (added {', '.join(sorted(caps - _BASELINE_CAPS))})")
    for sc in [psc] + [c.get("securityContext") or {} for c in conts]:
        if (sc.get("seccompProfile") or {}).get("type") == "Unconfined":
            out.append("seccompProfile (type Unconfined)")
            break
    if any((c.get("securityContext") or {}).get("procMount") not in (None, "Default") for c in conts):
        out.append("procMount (must be Default)")
    for sc in [psc] + [c.get("securityContext") or {} for c in conts]:
        se = sc.get("seLinuxOptions") or {}
        if se.get("user") or se.get("role"):
            out.append("seLinuxOptions (custom user or role)")
            break
    if level == "baseline":
        return out
    bad_vols = [v.get("name") for v in spec.get("volumes") or [] if not (set(v) - {"name"}) <= _RESTRICTED_VOLUMES]
    if bad_vols and not hp:
        out.append(f"restricted volume types (volumes {', '.join(map(str, bad_vols))})")
    for c in conts:
        sc = c.get("securityContext") or {}
        name = c.get("name")
        if sc.get("allowPrivilegeEscalation") is not False:
            out.append(f"allowPrivilegeEscalation != false (container {name} must set "
                       "securityContext.allowPrivilegeEscalation=false)")
        non_root = sc.get("runAsNonRoot", psc.get("runAsNonRoot"))
        if non_root is not True:
            out.append(f"runAsNonRoot != true (container {name} must set securityContext.runAsNonRoot=true)")
        if sc.get("runAsUser", psc.get("runAsUser")) == 0:
            out.append(f"runAsUser=0 (container {name} must not run as root)")
        cp = sc.get("capabilities") or {}
        if "ALL" not in (cp.get("drop") or []):
            out.append(f'unrestricted capabilities (container {name} must set securityContext.capabilities.drop=["ALL"])')
        if set(cp.get("add") or []) - {"NET_BIND_SERVICE"}:
            out.append(f"unrestricted capabilities (container {name} may only add NET_BIND_SERVICE)")
        prof = (sc.get("seccompProfile") or psc.get("seccompProfile") or {}).get("type")
        if prof not in ("RuntimeDefault", "Localhost"):
            out.append(f"seccompProfile (container {name} must set securityContext.seccompProfile.type to "
                       '"RuntimeDefault" or "Localhost")')
    return out


class PodSecurity:
    def _pod_security(self, pid: str, ns: str, name: str, pod: dict) -> list[str]:
        """Enforce the namespace's level (HttpError 403); the warnings of its warn level."""
        from .httpserver import HttpError
        from .objects import _key

        nso = self.store.get("namespaces", _key(pid, ns)) if self.store.keys("namespaces") else None
        labels = ((nso or {}).get("metadata") or {}).get("labels") or {}
        enforce, warn = labels.get(ENFORCE), labels.get(WARN)
        if not enforce and not warn:
            return []
        bad = violations(pod, enforce or "privileged")
        if bad:
            raise HttpError(403, f'pods "{name}" is forbidden: violates PodSecurity "{enforce}:latest": ' + "; ".join(bad))
        bad = violations(pod, warn or "privileged")
        return [f'would violate PodSecurity "{warn}:latest": ' + "; ".join(bad)] if bad else []
