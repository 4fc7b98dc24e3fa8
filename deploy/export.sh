#!/bin/bash
# Port-forward one Foremast endpoint to localhost (the reference ships one
# script per target under deploy/export/; here one script takes the target).
#   deploy/export.sh service     # REST API + dashboard   http://localhost:8099/dashboard/<ns>/<app>
#   deploy/export.sh brain       # brain exporter          http://localhost:8000/metrics (rank 0: every rank's gauges)
#   deploy/export.sh es          # Elasticsearch store     http://localhost:9200
#   deploy/export.sh prometheus  # Prometheus (kube-prometheus)  http://localhost:9090
#   deploy/export.sh grafana     # Grafana (kube-prometheus)     http://localhost:3000
#   deploy/export.sh example     # sidecar example app     http://localhost:8080
# Extra arguments go to kubectl (e.g. --context, --address 0.0.0.0).
set -euo pipefail
target=${1:-}
[ $# -gt 0 ] && shift
case "$target" in
  service)    exec kubectl --namespace foremast port-forward svc/foremast-service 8099 "$@" ;;
  brain)      exec kubectl --namespace foremast port-forward svc/foremast-brain 8000 "$@" ;;
  es)         exec kubectl --namespace foremast port-forward svc/elasticsearch 9200 "$@" ;;
  prometheus) exec kubectl --namespace monitoring port-forward svc/prometheus-k8s 9090 "$@" ;;
  grafana)    exec kubectl --namespace monitoring port-forward svc/grafana 3000 "$@" ;;
  example)    exec kubectl --namespace default port-forward svc/example-app 8080:80 "$@" ;;
  *) echo "usage: $0 {service|brain|es|prometheus|grafana|example} [kubectl args]" >&2; exit 2 ;;
esac
