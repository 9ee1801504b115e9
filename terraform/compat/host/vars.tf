# Inputs of the stock-Terraform host module: the same names setup writes into rancher.tf.

variable "hostname" {
  description = "machine name; also the node name in the control plane"
  type        = string
}

variable "networks" {
  description = "network ids (./tk8s networks); the first one provides the primary IP"
  type        = list(string)
}

variable "package" {
  description = "machine shape id or name (./tk8s packages); mi355x-<k>gpu owns k GPUs"
  type        = string
  default     = "mi355x-1gpu"
}

variable "root_authorized_keys" {
  description = "public key text authorised on the machine (never the private key)"
  type        = string
  default     = ""
}

variable "image" {
  description = "base image label; informational for the local provider"
  type        = string
  default     = "ubuntu-22.04-rocm-7.2"
}
