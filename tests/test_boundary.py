"""CPU: the drop-in boundary — registry, constructor kwargs, state-dict keys/shapes."""
import pytest
import torch

from tests.helpers import golden, reference_state_shapes


def test_registry_builds_by_class_and_by_name():
    from scflow_amd import MODELS
    from scflow_amd.decoder import SCFlowDecoder
    from tests.test_gpu_decoder import decoder_cfg
    a = MODELS.build(dict(type=SCFlowDecoder, **decoder_cfg()))
    b = MODELS.build(dict(type="SCFlowDecoder", **decoder_cfg()))
    assert type(a) is type(b) is SCFlowDecoder
    assert a.h_channels == 128 and a.cxt_channels == 128 and a.iters == 4
    with pytest.raises(KeyError):
        MODELS.build(dict(type="NoSuchDecoder"))


def test_state_dict_keys_and_shapes_match_reference():
    """Reference checkpoints load unchanged: identical keys and shapes."""
    from tests.test_gpu_decoder import build_decoder
    dec = build_decoder(4)
    ours = {k: tuple(v.shape) for k, v in dec.state_dict().items()}
    ref = dict(reference_state_shapes())
    assert set(ours) == set(ref)
    for k in ref:
        assert ours[k] == ref[k], k
    assert sum(v.numel() for v in dec.state_dict().values()) == 6_041_630


def test_load_state_dict_strict_roundtrip():
    from tests.test_gpu_decoder import build_decoder
    a = build_decoder(4, seed=0)
    b = build_decoder(4, seed=1)
    b.load_state_dict(a.state_dict(), strict=True)
    for (k, x), (_, y) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(x, y), k


def test_module_surface_matches_reference():
    from scflow_amd.modules import ConvGRU, CorrLookup, CorrelationPyramid, MotionEncoder, XHead
    assert CorrLookup(radius=4).r == 4
    assert CorrLookup(radius=4, align_corners=False).align_corners is False
    with pytest.raises(NotImplementedError):
        CorrLookup(radius=4, mode="nearest")
    assert CorrelationPyramid(num_levels=4).num_levels == 4
    me = MotionEncoder(num_levels=4, radius=4, net_type="Basic", act_cfg=dict(type="ReLU"))
    assert me.out_channels == [126]
    gru = ConvGRU(128, 256, "SeqConv")
    assert len(gru.conv_z) == 2 and gru.conv_z[0].conv.kernel_size == (1, 5)
    assert XHead(128, [256], 2, x="flow").predict_layer.kernel_size == (3, 3)


def _full_encoder_shapes(norm):
    g = golden("enc")
    return {str(k): tuple(int(x) for x in str(v).split(",") if x)
            for k, v in zip(g[f"keys_{norm}"], g[f"shapes_{norm}"])}


@pytest.mark.parametrize("norm", ["IN", "BN"])
def test_encoder_state_dict_matches_reference(norm):
    """RAFTEncoder (configs/refine_models/scflow_ycbv_real.py:179-206): same keys and shapes."""
    from scflow_amd import MODELS
    enc = MODELS.build(dict(type="RAFTEncoder", in_channels=3, out_channels=256, net_type="Basic",
                            norm_cfg=dict(type=norm)))
    ours = {k: tuple(v.shape) for k, v in enc.state_dict().items()}
    assert ours == _full_encoder_shapes(norm)


def test_refiner_builds_from_reference_config_blocks():
    """SCFlowRefiner with the config's encoder / context / decoder blocks; the feature encoder is
    shared (seperate_encoder=False) so checkpoint keys exist under both names."""
    from scflow_amd import MODELS
    from tests.test_gpu_decoder import decoder_cfg
    enc = dict(type="RAFTEncoder", in_channels=3, out_channels=256, net_type="Basic",
               norm_cfg=dict(type="IN"))
    ctx = dict(type="RAFTEncoder", in_channels=3, out_channels=256, net_type="Basic",
               norm_cfg=dict(type="BN"))
    r = MODELS.build(dict(type="SCFlowRefiner", cxt_channels=128, h_channels=128,
                          seperate_encoder=False, encoder=enc, cxt_encoder=ctx,
                          decoder=dict(type="SCFlowDecoder", **decoder_cfg()),
                          test_cfg=dict(iters=8)))
    assert r.real_encoder is r.render_encoder
    keys = set(r.state_dict())
    for k in _full_encoder_shapes("IN"):
        assert "real_encoder." + k in keys and "render_encoder." + k in keys
    for k in _full_encoder_shapes("BN"):
        assert "context." + k in keys
    assert r.test_iter_num == 8
