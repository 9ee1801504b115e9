# Inputs of the host module. Names match what setup writes into rancher.tf
# (hostname, networks, root_authorized_keys, package; image optional).

variable "hostname" { description = "machine name; also the node name in the control plane" }

variable "networks" {
  description = "network ids (./tk8s networks); the first one provides the primary IP"
  type        = "list"
}

variable "package" {
  description = "machine shape id or name (./tk8s packages); mi355x-<k>gpu owns k GPUs"
  default     = "mi355x-1gpu"
}

variable "root_authorized_keys" {
  description = "public key text authorised on the machine (never the private key)"
  default     = ""
}

variable "image" {
  description = "base image label; informational for the local provider"
  default     = "ubuntu-22.04-rocm-7.2"
}
