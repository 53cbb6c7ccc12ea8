"""``grpc.health.v1`` built in code (grpc_health is not installed in this image).

Same package/service/method names and field numbers as the standard health protocol the
reference registers (``services/risk/cmd/main.go:145-147``), so ``grpc_health_probe`` and
``grpcurl ... grpc.health.v1.Health/Check`` work against our server. (The standard
schema nests ``ServingStatus`` inside the response; it is top-level here, which is
identical on the wire.)
"""
from .builder import build_file, enum_values

FILE = "grpc/health/v1/health.proto"
SERVICE = "grpc.health.v1.Health"
M = build_file(
    FILE, "grpc.health.v1",
    {
        "HealthCheckRequest": [("service", 1, "string")],
        "HealthCheckResponse": [("status", 1, "enum:.grpc.health.v1.ServingStatus")],
    },
    enums={"ServingStatus": [("UNKNOWN", 0), ("SERVING", 1), ("NOT_SERVING", 2),
                             ("SERVICE_UNKNOWN", 3)]},
    services={"Health": [("Check", "HealthCheckRequest", "HealthCheckResponse"),
                         ("Watch", "HealthCheckRequest", "HealthCheckResponse", "server_stream")]},
)
STATUS = enum_values("grpc.health.v1.ServingStatus")
HealthCheckRequest = M["HealthCheckRequest"]
HealthCheckResponse = M["HealthCheckResponse"]
