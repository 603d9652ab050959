"""The gRPC front end of secure_aggregation/app/src/server.rs (:217-256), in Python.

Serves service `secure_aggregation.Aggregator` (proto/secure_aggregation.proto:4-7)
with methods Aggregate and Start on 0.0.0.0:50051 by default, the reference
server's address, so src/fl_main.py / src/proto_client.py (ADDRESS 127.0.0.1:50051)
connect to it unchanged.  Messages are (de)serialised by fltee.wire (no generated
code); the handlers are fltee.server.Aggregator, the server.rs logic over the C ABI.

    python -m fltee.grpc_server [--address 0.0.0.0:50051] [--device 0] [--dp]
                                [--strict-reference] [--quiet]

Like the reference: verbose on, dp off (server.rs:236-237; --dp turns DP on for
the configs[3] runs), one enclave per process; calls are serialised by the
library's process-wide lock (the enclave's single TCS).  A handler panic in
tonic fails that RPC; here ServerPanic aborts it with StatusCode.INTERNAL.
The receive limit is raised to 2 GiB - 1 (tonic's 4 MiB default would refuse
configs[4]-sized uploads; the unchanged client never sends more than that).
"""
import argparse
import sys
import time
from concurrent import futures

import grpc

from . import wire
from .server import Aggregator, ServerPanic

SERVICE = "secure_aggregation.Aggregator"
MAX_MESSAGE = 2**31 - 1


class AggregatorService:
    def __init__(self, aggregator, verbose=True):
        self.agg = aggregator
        self.verbose = verbose

    def Aggregate(self, req, context):
        if self.verbose:
            print(f"[Server] Aggregate fl_id={req['fl_id']} round={req['round']} "
                  f"alg={req['aggregation_alg']} clients={len(req['client_ids'])} "
                  f"bytes={len(req['encrypted_parameters'])}", flush=True)
        try:
            r = self.agg.aggregate(req["fl_id"], req["round"], req["encrypted_parameters"],
                                   req["num_of_parameters"], req["num_of_sparse_parameters"],
                                   req["optimal_num_of_clients"], req["aggregation_alg"],
                                   req["client_ids"])
        except ServerPanic as e:
            context.abort(grpc.StatusCode.INTERNAL, str(e))
        return r

    def Start(self, req, context):
        if self.verbose:
            print(f"[Server] Start fl_id={req['fl_id']} clients={len(req['client_ids'])} "
                  f"alg={req['aggregation_alg']} d={req['num_of_parameters']}", flush=True)
        try:
            return self.agg.start(req["fl_id"], req["client_ids"], req["sigma"], req["clipping"],
                                  req["alpha"], req["sampling_ratio"], req["aggregation_alg"],
                                  req["num_of_parameters"], req["num_of_sparse_parameters"])
        except ServerPanic as e:
            context.abort(grpc.StatusCode.INTERNAL, str(e))


def make_server(aggregator, address="0.0.0.0:50051", verbose=True, max_workers=4):
    """Returns (grpc.Server, bound port).  Port 0 picks a free port."""
    svc = AggregatorService(aggregator, verbose)
    handlers = {
        "Aggregate": grpc.unary_unary_rpc_method_handler(
            svc.Aggregate, request_deserializer=wire.decode_aggregate_request,
            response_serializer=wire.encode_aggregate_response),
        "Start": grpc.unary_unary_rpc_method_handler(
            svc.Start, request_deserializer=wire.decode_start_request,
            response_serializer=wire.encode_start_response),
    }
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers),
                         options=[("grpc.max_receive_message_length", MAX_MESSAGE),
                                  ("grpc.max_send_message_length", MAX_MESSAGE)])
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))
    port = server.add_insecure_port(address)
    if port == 0:
        raise RuntimeError(f"cannot bind {address}")
    return server, port


class Client:
    """The stub src/proto_client.py gets from secure_aggregation_pb2_grpc, over fltee.wire
    (used by the tests and by drivers that do not have the generated pb2)."""

    def __init__(self, address, max_message=MAX_MESSAGE):
        self.channel = grpc.insecure_channel(
            address, options=[("grpc.max_receive_message_length", max_message),
                              ("grpc.max_send_message_length", max_message)])
        self._agg = self.channel.unary_unary(f"/{SERVICE}/Aggregate",
                                             request_serializer=wire.encode_aggregate_request,
                                             response_deserializer=wire.decode_aggregate_response)
        self._start = self.channel.unary_unary(f"/{SERVICE}/Start",
                                               request_serializer=wire.encode_start_request,
                                               response_deserializer=wire.decode_start_response)

    def Aggregate(self, **fields):
        return self._agg(fields)

    def Start(self, **fields):
        return self._start(fields)

    def close(self):
        self.channel.close()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--address", default="0.0.0.0:50051")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--dp", action="store_true", help="DP noise on (server.rs:237 forces off)")
    ap.add_argument("--strict-reference", action="store_true",
                    help="apply server.rs:126-128's optimal_num_of_clients check to every alg")
    ap.add_argument("--quiet", action="store_true")
    args = ap.parse_args(argv)
    agg = Aggregator(device=args.device, verbose=not args.quiet, dp=args.dp,
                     strict_reference=args.strict_reference)
    server, port = make_server(agg, args.address, verbose=not args.quiet)
    server.start()
    print(f"[Server] Now GRPC Server is binded on {args.address} (port {port})", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        server.stop(0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
