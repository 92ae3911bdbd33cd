# k8s-watcher-amd — container image (SURVEY §2.2: the reference claims
# "Dockerized" but ships no Dockerfile).
FROM python:3.10-slim AS build
RUN apt-get update && apt-get install -y --no-install-recommends g++ libssl-dev zlib1g-dev && rm -rf /var/lib/apt/lists/*
WORKDIR /app
COPY requirements.txt ./
COPY k8s_watcher_amd/ k8s_watcher_amd/
RUN pip install --no-cache-dir -r requirements.txt && python -m k8s_watcher_amd.ops.native

FROM python:3.10-slim
# runtime: libssl3 (the notifier core runs TLS itself) ships in the slim image
WORKDIR /app
COPY requirements.txt ./
RUN pip install --no-cache-dir -r requirements.txt \
 && useradd --uid 10001 --no-create-home watcher
COPY --from=build /app/k8s_watcher_amd/ k8s_watcher_amd/
COPY main.py ./
COPY watcher/ watcher/
COPY config/ config/
USER 10001
ENV PYTHONUNBUFFERED=1
EXPOSE 9090
ENTRYPOINT ["python", "main.py"]
CMD ["production"]
