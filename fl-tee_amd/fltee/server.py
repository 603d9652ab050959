"""The Aggregator service logic of secure_aggregation/app/src/server.rs, over the C ABI.

`Aggregator.start` / `Aggregator.aggregate` take and return exactly the fields of
proto/secure_aggregation.proto's StartRequestParameters / AggregateRequestParameters
(and the response messages), so a gRPC front end only has to (de)serialise.  Where
server.rs panics, these raise `ServerPanic` (a tonic handler panic aborts the
request).  Documented deviations from the reference host:

  * server.rs:126-128 rejects `optimal_num_of_clients > |client_ids|` for EVERY
    algorithm, which kills fl_main.py's defaults (n=30 < 100) for algs 1-5.  The
    check is applied only when aggregation_alg == 6 (`strict_reference=True`
    restores the reference behaviour).
  * server.rs:237 hard-wires dp = false; here it is a constructor argument.
"""
import time

from . import _lib as L
from .ecalls import Enclave


class ServerPanic(RuntimeError):
    pass


class Aggregator:
    def __init__(self, device=0, verbose=False, dp=False, strict_reference=False, enclave=None):
        self.enclave = enclave if enclave is not None else Enclave(device)
        self.verbose = verbose
        self.dp = dp
        self.strict_reference = strict_reference

    # server.rs:44-108
    def start(self, fl_id, client_ids, sigma, clipping, alpha, sampling_ratio, aggregation_alg,
              num_of_parameters, num_of_sparse_parameters):
        st, rv = self.enclave.ecall_fl_init(fl_id, client_ids, num_of_parameters,
                                            num_of_sparse_parameters, sigma, clipping, alpha,
                                            sampling_ratio, aggregation_alg, self.verbose, self.dp)
        if st != L.SUCCESS or rv != L.SUCCESS:
            raise ServerPanic("Error at ecall_fl_init")
        import numpy as np
        sample_size = int(np.float32(sampling_ratio) * np.float32(len(client_ids)))  # f32 then as usize
        st, rv, sampled = self.enclave.ecall_start_round(fl_id, 0, sample_size)
        if st != L.SUCCESS or rv != L.SUCCESS:
            raise ServerPanic("Error at ecall_start_round")
        return dict(fl_id=fl_id, round=0, client_ids=[int(x) for x in sampled])

    # server.rs:111-215
    def aggregate(self, fl_id, round, encrypted_parameters, num_of_parameters,
                  num_of_sparse_parameters, optimal_num_of_clients, aggregation_alg, client_ids):
        if optimal_num_of_clients > len(client_ids) and (self.strict_reference or aggregation_alg == 6):
            raise ServerPanic(f"optimal_num_of_clients is more than client size {len(client_ids)}")
        t0 = time.perf_counter()
        if aggregation_alg == 6:
            st, rv, out, times = self.enclave.ecall_client_size_optimized_secure_aggregation(
                fl_id, round, optimal_num_of_clients, client_ids, encrypted_parameters,
                num_of_parameters, num_of_sparse_parameters, aggregation_alg)
            if st != L.SUCCESS or rv != L.SUCCESS:
                raise ServerPanic("Error at ecall_client_size_optimized_secure_aggregation")
        else:
            st, rv, out, times = self.enclave.ecall_secure_aggregation(
                fl_id, round, client_ids, encrypted_parameters, num_of_parameters,
                num_of_sparse_parameters, aggregation_alg)
            if st != L.SUCCESS or rv != L.SUCCESS:
                raise ServerPanic("Error at ecall_secure_aggregation")
        elapsed = time.perf_counter() - t0
        # "Assuming that the next round is the same number of participants." (server.rs:188)
        st, rv, sampled = self.enclave.ecall_start_round(fl_id, round + 1, len(client_ids))
        if st != L.SUCCESS or rv != L.SUCCESS:
            raise ServerPanic("[Server] Error at ecall_start_round")
        return dict(updated_parameters=out, execution_time=float(elapsed),
                    client_ids=[int(x) for x in sampled], round=round + 1,
                    enclave_times=times)
