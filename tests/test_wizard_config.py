"""Wizard prompts/validation (setup.sh:94-483) and the ./config file (setup.sh:199-254, 543-549)."""
import io

import pytest

from tritonk8ssupervisor_amd import wizard as wz
from tritonk8ssupervisor_amd.config import (ClusterConfig, KEY_ORDER, config_from_dict, export_vars,
                                            parse_config_text, read_config, render_config, write_config)
from tritonk8ssupervisor_amd.provider.local import LocalProvider


@pytest.fixture
def prov(tmp_path, monkeypatch):
    monkeypatch.setenv("TK8S_FAKE_GPUS", "8")
    return LocalProvider(tmp_path / ".tk8s")


# ---- validation tables: one row per reference regex ---------------------------------
@pytest.mark.parametrize("s,ok", [
    ("kubemaster", True), ("k8", True), ("Master01", True), ("a", False), ("1master", False),
    ("kube-master", False), ("kube_master", False), ("", False), ("kube master", False), ("ab9Z", True),
])
def test_hostname_rule(s, ok):  # setup.sh:276, 288: ^[a-zA-Z][0-9a-zA-Z]+$
    assert wz.valid_hostname(s) is ok


@pytest.mark.parametrize("s,ok", [("1", True), ("9", True), ("0", False), ("10", False), ("-1", False),
                                  ("", False), ("a", False), (" 2", False)])
def test_node_count_rule(s, ok):  # setup.sh:301: ^[1-9]$ — HARD LIMIT 1-9 nodes
    assert wz.valid_node_count(s) is ok


@pytest.mark.parametrize("s,count,want", [
    ("1", 3, [1]), ("1,3", 3, [1, 3]), ("4", 3, None), ("0", 3, None), ("1,,2", 3, None),
    ("99", 99, [99]), ("100", 120, None), ("a", 3, None), ("1,2,", 3, None),
])
def test_index_list_rule(s, count, want):  # setup.sh:337-345, 380
    assert wz.parse_index_list(s, count) == want


def test_normalize_list_sort_uniq():  # setup.sh:333-334 tr | sort | uniq | tr
    assert wz.normalize_list("3,1,3,2") == "1,2,3"
    assert wz.normalize_list('"b,a"') == "a,b"
    assert wz.normalize_list("") == ""


@pytest.mark.parametrize("s,ok", [("1", True), ("12", True), ("0", False), ("1,2", False), ("", False)])
def test_package_rule(s, ok):  # setup.sh:428
    assert bool(wz.PACKAGE_RE.match(s)) is ok


# ---- getArgument ----------------------------------------------------------------------
def test_get_argument_default_and_override():
    out = io.StringIO()
    p = wz.Prompter(out=out, answers=["", "custom"])
    assert p.get_argument("Name:", "k8s dev") == "k8s dev"
    assert p.get_argument("Name:", "k8s dev") == "custom"
    assert "Name: (k8s dev) " in out.getvalue()


def test_get_argument_without_default_reprompts_instead_of_looping_forever():
    # reference W2 bug: no `break` when there is no default (setup.sh:98-99)
    p = wz.Prompter(out=io.StringIO(), answers=["", "  ", "x"])
    assert p.get_argument("Q:") == "x"


def test_prompter_eof_is_an_error_not_a_hang():
    p = wz.Prompter(inp=io.StringIO(""), out=io.StringIO())
    with pytest.raises(EOFError):
        p.get_argument("Q:", "d")


# ---- whole wizard ---------------------------------------------------------------------
def test_wizard_defaults_match_reference(prov):
    cfg = ClusterConfig()
    out = io.StringIO()
    wz.run_wizard(cfg, prov, answers={}, out=out)
    assert cfg.KUBERNETES_NAME == "k8s dev" and cfg.KUBERNETES_DESCRIPTION == "k8s dev"
    assert cfg.RANCHER_MASTER_HOSTNAME == "kubemaster"
    assert cfg.KUBERNETES_NODE_HOSTNAME_BEGINSWITH == "kubenode"
    assert cfg.KUBERNETES_NUMBER_OF_NODES == 1
    pub = prov.network_by_id_or_name("local-public").id
    assert cfg.RANCHER_MASTER_NETWORKS == pub and cfg.KUBERNETES_NODE_NETWORKS == pub
    assert cfg.HOST_PACKAGE == prov.package_by_id_or_name("mi355x-1gpu").id
    text = out.getvalue()
    # prompt order of setup.sh:265-449
    order = ["Name your Kubernetes environment:", "Describe this Kubernetes environment:", "Hostname of the master:",
             "Enter a string to use for appending", "How many nodes", "What networks should the master",
             "What networks should the nodes", "What KVM package", "Is the above config correct"]
    pos = [text.index(s) for s in order]
    assert pos == sorted(pos)


def test_wizard_description_defaults_to_name(prov):
    cfg = ClusterConfig(KUBERNETES_DESCRIPTION="")
    wz.run_wizard(cfg, prov, answers={"name": "gpu lab"}, out=io.StringIO())
    assert cfg.KUBERNETES_DESCRIPTION == "gpu lab"


def test_wizard_reprompts_on_invalid_answers(prov):
    cfg = ClusterConfig()
    # bad hostname, good; bad prefix, good; bad count x2, good; bad nets, good; good; bad pkg, good; confirm junk, yes
    script = ["env", "", "1bad", "boss", "no-dash", "wk", "0", "12", "4", "9", "2,1", "", "77", "3", "maybe", "yes"]
    out = io.StringIO()
    p = wz.Prompter(out=out, answers=script)
    wz.get_config_from_user(cfg, prov, p)
    wz.verify_config(cfg, p)
    assert cfg.RANCHER_MASTER_HOSTNAME == "boss" and cfg.KUBERNETES_NODE_HOSTNAME_BEGINSWITH == "wk"
    assert cfg.KUBERNETES_NUMBER_OF_NODES == 4
    nets = prov.networks()
    assert cfg.RANCHER_MASTER_NETWORKS == f"{nets[0].id},{nets[1].id}"
    assert cfg.HOST_PACKAGE == prov.packages()[2].id
    text = out.getvalue()
    assert text.count("Must start with a letter") == 2
    assert "number between 1-9" in text
    assert "Values should be comma separated between 1 and 3" in text
    assert "Value should be between 1 and 5" in text
    assert "Please answer yes or no." in text
    assert p.answers == []


def test_wizard_no_aborts_with_exit_zero(prov):
    with pytest.raises(wz.WizardAbort) as ei:
        wz.run_wizard(ClusterConfig(), prov, answers={"confirm": "no"}, out=io.StringIO())
    assert ei.value.code == 0


def test_answers_by_name_and_index(prov):
    script = wz.answers_to_script({"nodes": 8, "package": "mi355x-1gpu", "master_networks": ["local-fabric", "local-public"],
                                   "node_networks": "2"}, prov)
    assert script[4] == "8"
    assert script[5] == "1,2" and script[6] == "2"
    assert script[7] == str([p.name for p in prov.packages()].index("mi355x-1gpu") + 1)
    with pytest.raises(ValueError):
        wz.answers_to_script({"package": "k4-highcpu-kvm-7.75G"}, prov)


def test_answers_cannot_bypass_validation(prov):
    with pytest.raises(EOFError):  # 10 nodes is rejected; the scripted run then runs out of answers
        wz.run_wizard(ClusterConfig(), prov, answers={"nodes": 10}, out=io.StringIO())


def test_load_answers_yaml_json_list(tmp_path):
    (tmp_path / "a.yaml").write_text("nodes: 4\npackage: mi355x-1gpu\n")
    (tmp_path / "b.json").write_text('{"nodes": 2}')
    (tmp_path / "c.yaml").write_text("- env\n- desc\n")
    assert wz.load_answers(str(tmp_path / "a.yaml")) == {"nodes": 4, "package": "mi355x-1gpu"}
    assert wz.load_answers(str(tmp_path / "b.json")) == {"nodes": 2}
    assert wz.load_answers(str(tmp_path / "c.yaml")) == {"name": "env", "description": "desc"}


# ---- config file -----------------------------------------------------------------------
def test_config_round_trip(tmp_path):
    cfg = ClusterConfig(SDC_URL="local://h", SDC_ACCOUNT="me", SDC_KEY_ID="aa:bb", SDC_KEY="/k/id",
                        RANCHER_MASTER_NETWORKS="n1", KUBERNETES_NODE_NETWORKS="n1,n2", KUBERNETES_NUMBER_OF_NODES=8,
                        KUBERNETES_NAME="k8s dev", KUBERNETES_DESCRIPTION='with "quotes"', HOST_PACKAGE="p")
    cfg.extra["CUSTOM"] = "1"
    write_config(tmp_path / "config", cfg)
    text = (tmp_path / "config").read_text()
    assert text.splitlines()[0] == "ANSIBLE_HOST_KEY_CHECKING=False"  # setup.sh:253 writes it first
    assert 'KUBERNETES_NAME="k8s dev"' in text and "KUBERNETES_NUMBER_OF_NODES=8" in text
    back = read_config(tmp_path / "config")
    assert back.KUBERNETES_NUMBER_OF_NODES == 8 and back.KUBERNETES_NODE_NETWORKS == "n1,n2"
    assert back.KUBERNETES_DESCRIPTION == "with quotes"  # quotes stripped like setup.sh:450
    assert back.extra == {"CUSTOM": "1"}
    assert [l.split("=")[0] for l in text.splitlines()][:len(KEY_ORDER)] == KEY_ORDER


def test_parse_config_drops_blank_lines_and_quotes():  # exportVars setup.sh:543-549
    kv = parse_config_text('\nA=1\n\nB="two words"\n# c\nC=\'x\'\n')
    assert kv == {"A": "1", "B": "two words", "C": "x"}


def test_export_vars_reaches_environment():
    env = {}
    export_vars(config_from_dict({"KUBERNETES_NAME": "x", "KUBERNETES_NUMBER_OF_NODES": "3"}), env)
    assert env["ANSIBLE_HOST_KEY_CHECKING"] == "False"  # reaches ansible this way (setup.sh:253)
    assert env["KUBERNETES_NAME"] == "x" and env["KUBERNETES_NUMBER_OF_NODES"] == "3"


def test_node_names():
    cfg = ClusterConfig(KUBERNETES_NODE_HOSTNAME_BEGINSWITH="kubenode", KUBERNETES_NUMBER_OF_NODES=3)
    assert cfg.node_names() == ["kubenode1", "kubenode2", "kubenode3"]
    assert render_config(cfg).count("\n") == len(KEY_ORDER)
