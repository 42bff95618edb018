"""Drop-in mirror of the reference package layout (HIP-backed hot path).

`pkgutil.extend_path` appends every other `<sys.path entry>/<this package>` directory to
`__path__`: with this package ahead of the reference on sys.path the modules shipped here
(training, models_pytorch, privacy, models, interfaces, validation, fedavg) shadow the
reference's, and every module not shipped here (coordinator, compression, data_loader,
grpc_utils, convergence, ...) still resolves from the reference tree.
"""
from pkgutil import extend_path

__path__ = extend_path(__path__, __name__)
