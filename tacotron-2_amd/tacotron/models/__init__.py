"""tacotron.models.create_model (code/tacotron/models/__init__.py:5-11)."""
from .tacotron import Tacotron


def create_model(name, hparams):
    if name == 'Tacotron':
        return Tacotron(hparams)
    elif name == 'Tacotron_emt_attn':
        raise NotImplementedError(
            "Tacotron_emt_attn (tacotron_emt_attn.py, --emt_attn) is not on the MI355X path yet")
    else:
        raise Exception('Unknown model: ' + name)
