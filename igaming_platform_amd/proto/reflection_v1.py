"""``grpc.reflection.v1alpha`` / ``v1`` messages built in code (grpcio-reflection is not in the
image). The reference registers reflection (services/risk/cmd/main.go:150) so grpcurl works
without .proto files (Makefile:231-241); so does this server."""
from .builder import build_file

PKGS = ("grpc.reflection.v1alpha", "grpc.reflection.v1")


def _schema():
    return {
        "ServerReflectionRequest": [
            ("host", 1, "string"), ("file_by_filename", 3, "string"), ("file_containing_symbol", 4, "string"),
            ("all_extension_numbers_of_type", 6, "string"), ("list_services", 7, "string"),
        ],
        "FileDescriptorResponse": [("file_descriptor_proto", 1, "bytes", "rep")],
        "ExtensionNumberResponse": [("base_type_name", 1, "string"), ("extension_number", 2, "int32", "rep")],
        "ServiceResponse": [("name", 1, "string")],
        "ListServiceResponse": [("service", 1, "{pkg}.ServiceResponse", "rep")],
        "ErrorResponse": [("error_code", 1, "int32"), ("error_message", 2, "string")],
        "ServerReflectionResponse": [
            ("valid_host", 1, "string"), ("original_request", 2, "{pkg}.ServerReflectionRequest"),
            ("file_descriptor_response", 4, "{pkg}.FileDescriptorResponse"),
            ("all_extension_numbers_response", 5, "{pkg}.ExtensionNumberResponse"),
            ("list_services_response", 6, "{pkg}.ListServiceResponse"),
            ("error_response", 7, "{pkg}.ErrorResponse"),
        ],
    }


def build(pkg: str):
    sch = {}
    for m, flds in _schema().items():
        sch[m] = [tuple(x.replace("{pkg}", "." + pkg) if isinstance(x, str) else x for x in f) for f in flds]
    return build_file(pkg.replace(".", "/") + "/reflection.proto", pkg, sch,
                      services={"ServerReflection": [("ServerReflectionInfo", "ServerReflectionRequest",
                                                      "ServerReflectionResponse", "bidi")]})


M = {pkg: build(pkg) for pkg in PKGS}
