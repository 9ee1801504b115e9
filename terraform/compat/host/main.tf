# Stock-Terraform form of one host machine (terraform >= 1.4): the built-in terraform_data
# resource, no provider to download. Its provisioners call the tk8s provider CLI, so
#   cd terraform && terraform init && terraform plan && terraform apply
# creates and destroys the same machines the in-repo engine does with resource tk8s_machine
# (terraform/host/main.tf). The engine reads this form too (provision.py: terraform_data with
# these `input` keys plans exactly like tk8s_machine) and creates the machine through its fast
# path instead of running the CLI provisioners.
resource "terraform_data" "host" {
  input = {
    name                 = "${var.hostname}"
    package              = "${var.package}"
    image                = "${var.image}"
    networks             = "${var.networks}"
    root_authorized_keys = "${var.root_authorized_keys}"
    tags = {
      name = "${var.hostname}"
      role = "host"
    }
  }

  # Create the machine, bootstrap-check it and append its IP for Ansible (setup.sh's masters.ip /
  # hosts.ip hand-off).
  provisioner "local-exec" {
    command = "../tk8s --workdir .. machine create --name ${self.input.name} --package ${self.input.package} --networks ${join(",", self.input.networks)} --role host --ip-file hosts.ip"
  }

  provisioner "local-exec" {
    when    = destroy
    command = "../tk8s --workdir .. machine delete --name ${self.input.name}"
  }
}
