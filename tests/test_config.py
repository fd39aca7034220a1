"""INI config parity with the reference typing rules (auxiliary_functions.py:387-438)."""
import os
import textwrap

from gfedntm_amd.utils.config import (DEFAULT_GRADS_TO_SHARE, load_config,
                                      model_kwargs_from_params, read_config_experiments)


def test_default_config_typing():
    cfg = load_config()
    p = cfg.training_params
    assert p["n_components"] == 50 and isinstance(p["n_components"], int)
    assert p["hidden_sizes"] == (50, 50)
    assert p["lr"] == 0.002 and isinstance(p["lr"], float)
    assert p["momentum"] == 0.99
    assert p["learn_priors"] is True and p["reduce_on_plateau"] is False
    assert p["labels"] == "" and p["topic_prior_variance"] is None
    assert p["model_type"] == "prodLDA" and p["solver"] == "adam"
    assert cfg.grpc_max_message_length == 262144000
    assert cfg.grads_to_share == DEFAULT_GRADS_TO_SHARE and len(cfg.grads_to_share) == 22
    assert cfg.server_port == 50051 and cfg.time_termination == 604800


def test_custom_ini(tmp_path):
    f = tmp_path / "c.cf"
    f.write_text(textwrap.dedent("""
        [ntms]
        n_components = 7
        hidden_sizes = (20, 30, 40)
        learn_priors = False
        dropout = 0.1
        model_type = LDA
        labels = something
        topic_prior_variance = 0.5
        [save_dir]
        save_client = out/c
    """))
    p = read_config_experiments(str(f))
    assert p["n_components"] == 7 and p["hidden_sizes"] == (20, 30, 40)
    assert p["learn_priors"] is False and p["dropout"] == 0.1
    assert p["labels"] == "" and p["topic_prior_variance"] is None   # reference quirks
    kw = model_kwargs_from_params(p)
    assert kw["model_type"] == "LDA" and "labels" not in kw
    cfg = load_config(str(f))
    assert cfg.save_client == "out/c"
    assert cfg.resolve("out/c", "/w") == "/w/out/c"


def test_grpc_options():
    cfg = load_config()
    keys = dict(cfg.grpc_client_options())
    assert keys["grpc.max_send_message_length"] == 262144000
    srv = dict(cfg.grpc_server_options())
    assert srv["grpc.keepalive_time_ms"] == 10000 and srv["grpc.http2.max_ping_strikes"] == 0


def test_cli_accepts_reference_readme_syntax():
    """README.md:77 writes `main.py start_client --id <id> ...`; the role word is accepted."""
    import pytest
    from gfedntm_amd.cli import build_parser, main
    a = build_parser().parse_args(["start_client", "--id", "2", "--data_type", "real", "--fos", "x"])
    assert a.command == "start_client" and a.id == 2
    assert build_parser().parse_args(["--id", "0"]).command is None
    with pytest.raises(SystemExit):
        main(["start_client", "--id", "0"])


def test_matmul_dtype_knob(tmp_path):
    """[amd] matmul_dtype reaches the model kwargs; fp32 (the reference's precision) is the
    default and adds nothing."""
    from gfedntm_amd.utils.config import load_config, model_kwargs_from_params
    assert "matmul_dtype" not in load_config().training_params
    src = open(os.path.join(os.path.dirname(__file__), "..", "config", "dft_params.cf")).read()
    p = tmp_path / "bf16.cf"
    p.write_text(src.replace("matmul_dtype = fp32", "matmul_dtype = bf16"))
    cfg = load_config(str(p))
    assert model_kwargs_from_params(cfg.training_params)["matmul_dtype"] == "bf16"
